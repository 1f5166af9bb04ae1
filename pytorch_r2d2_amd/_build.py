"""In-tree build of the native code for gfx950 (MI355X).

Two shared objects are produced next to this file (git-ignored, they travel to the GPU box
with the source snapshot):

* ``_r2d2_kernels.so`` -- every HIP kernel in ``csrc/kernels/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` with a plain ``extern "C"`` launcher ABI (raw device pointers +
  ``hipStream_t``).  No torch headers: kernels compile in seconds and the launchers are safe
  under HIP-graph stream capture (no allocation, no synchronisation).
* ``_r2d2_runtime.so`` -- the host-side C++ runtime (``csrc/runtime/*.cpp``): shared-memory
  SPSC trajectory rings, the sum-tree CPU mirror, fcntl file locks, the supervisor heartbeat
  table.  Plain C++17, C ABI.

Both are loaded with ``ctypes`` *after* ``import torch`` so that ``libamdhip64.so.7`` resolves
to the HIP runtime torch already mapped (one HIP runtime per process).

Usage: ``python -m pytorch_r2d2_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
KERNEL_SO = PKG / "_r2d2_kernels.so"
RUNTIME_SO = PKG / "_r2d2_runtime.so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-Wno-unused-variable"]
if os.environ.get("R2D2_PROBES"):
    # the LSTM kernels' clock-stamp hooks (csrc/lstm_common.h PL_PROBE): probe builds only
    HIP_FLAGS.append("-DR2_LSTM_PROBES=1")
CXX = os.environ.get("CXX", "g++")
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]


def _digest(paths) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(Path(p).name.encode())
        h.update(Path(p).read_bytes())
    h.update(" ".join(HIP_FLAGS + CXX_FLAGS).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}")
    return r.stdout


def _build_so(srcs, out: Path, compiler, flags, link_extra, jobs: int, force: bool):
    headers = list(CSRC.glob("*.h")) + list((CSRC / "runtime").glob("*.h"))
    stamp = out.with_suffix(".so.stamp")
    digest = _digest(list(srcs) + headers)
    if not force and out.exists() and stamp.exists() and stamp.read_text().strip() == digest:
        return False
    BUILD.mkdir(exist_ok=True)
    objs = []
    cmds = []
    for s in srcs:
        o = BUILD / (s.stem + (".hip.o" if s.suffix == ".hip" else ".cpp.o"))
        objs.append(o)
        cmds.append([compiler, *flags, "-I", str(CSRC), "-c", str(s), "-o", str(o)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, cmds))
    tmp = out.with_suffix(".so.tmp")
    _run([compiler, *flags, "-shared", "-o", str(tmp), *map(str, objs), *link_extra])
    os.replace(tmp, out)
    stamp.write_text(digest)
    return True


def build_runtime(force: bool = False, jobs: int = 0) -> bool:
    """Host runtime only (g++; used on machines without a ROCm toolchain)."""
    rt_srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    return _build_so(rt_srcs, RUNTIME_SO, CXX, CXX_FLAGS, ["-lpthread", "-lrt"],
                     jobs or min(8, os.cpu_count() or 4), force)


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> None:
    jobs = jobs or min(8, os.cpu_count() or 4)
    if not Path(HIPCC).exists() and shutil.which("hipcc") is None:
        raise RuntimeError("hipcc not found; ROCm toolchain required to build gfx950 kernels")
    hip_srcs = sorted((CSRC / "kernels").glob("*.hip"))
    k = _build_so(hip_srcs, KERNEL_SO, HIPCC, HIP_FLAGS, [], jobs, force)
    rt_srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    r = False
    if rt_srcs:
        r = _build_so(rt_srcs, RUNTIME_SO, CXX, CXX_FLAGS, ["-lpthread", "-lrt"], jobs, force)
    if verbose:
        print(f"[r2d2 build] kernels: {'rebuilt' if k else 'up to date'} -> {KERNEL_SO.name}; "
              f"runtime: {'rebuilt' if r else 'up to date'} -> {RUNTIME_SO.name}")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    main()
