"""Variance of the DP two-level prioritized sampling (parallel/sharded_replay.py) vs one merged
replay and vs multinomial shard counts, over shard imbalance, by Monte Carlo (CPU).

    python tools/dp_sampling_variance.py > profiles/r03_dp_sampling_variance.txt
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_r2d2_amd.parallel.sharded_replay import imbalance_factor, mc_estimator_variance  # noqa: E402


def main():
    W, M, B = 8, 256, 16
    print(f"# W={W} shards x {M} sequences, B={B} per rank, 4000 trials per row; f ~ N(0,1) per sequence")
    print("# spread = shard priority totals scaled by 1 + spread * u, u in [-1, 1] evenly over shards")
    print("# columns: spread, imbalance W*sum s_k^2, var ratio local_ratio/merged, multinomial/merged, "
          "bias(local_ratio) in units of its std error")
    for spread in (0.0, 0.1, 0.25, 0.5, 0.9):
        g = np.random.default_rng(1)
        scale = 1 + spread * np.linspace(-1, 1, W)
        pr = [(g.random(M) + 0.05) * scale[k] for k in range(W)]
        fv = [g.normal(size=M) for _ in range(W)]
        res, mu = mc_estimator_variance(pr, fv, B)
        stats = torch.tensor([[p.sum(), M, 0.0] for p in pr], dtype=torch.float64)
        imb = float(imbalance_factor(stats))
        vm = res["merged"][1]
        bias = (res["local_ratio"][0] - mu) / np.sqrt(res["local_ratio"][1] / 4000)
        print(f"{spread:5.2f}  {imb:6.3f}  {res['local_ratio'][1] / vm:6.3f}  "
              f"{res['multinomial'][1] / vm:6.3f}  {bias:+5.2f}")


if __name__ == "__main__":
    main()
