"""Checkpointing.

* Reference format (``/root/reference/learner.py:117-120``): ``save/{n_epochs}_save.pt`` =
  ``torch.save`` of the CPU state_dict of the online net with the 18 reference keys.  Loads with
  ``torch.load(weights_only=True)`` in both frameworks.  Fix Q11: the directory is created.
* Full state (absent in the reference): online + target weights, optimizer state,
  step counters, RNG states and the config, written atomically; ``load_full_checkpoint`` +
  ``Learner``/engine ``resume`` continue training bit-for-bit from it.
"""
from __future__ import annotations

import dataclasses
import json
import os
import tempfile
from typing import Any, Dict, Optional

import numpy as np
import torch


def _atomic_save(obj, path: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, suffix=".tmp")
    os.close(fd)
    try:
        torch.save(obj, tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def reference_checkpoint_path(n_epochs: int, save_dir: str = "save") -> str:
    return os.path.join(save_dir, f"{n_epochs}_save.pt")


def save_reference_checkpoint(state_dict: Dict[str, torch.Tensor], n_epochs: int,
                              save_dir: str = "save") -> str:
    path = reference_checkpoint_path(n_epochs, save_dir)
    _atomic_save({k: v.detach().cpu().clone() for k, v in state_dict.items()}, path)
    return path


def load_reference_checkpoint(path: str) -> Dict[str, torch.Tensor]:
    """Load a reference-format checkpoint (ours or the reference's) without unpickling code."""
    return torch.load(path, map_location="cpu", weights_only=True)


def save_full_checkpoint(path: str, online_sd, target_sd, optimizer_state, step: int, cfg=None,
                         extra: Optional[Dict[str, Any]] = None) -> str:
    obj = {
        "format": "pytorch_r2d2_amd.full.v1",
        "online": {k: v.detach().cpu().clone() for k, v in online_sd.items()},
        "target": {k: v.detach().cpu().clone() for k, v in target_sd.items()},
        "optimizer": optimizer_state,
        "step": int(step),
        "config_json": json.dumps(dataclasses.asdict(cfg)) if cfg is not None else "{}",
        "torch_rng": torch.get_rng_state(),
        "numpy_rng_json": json.dumps(_np_state()),
        "extra": extra or {},
    }
    _atomic_save(obj, path)
    return path


def _np_state():
    s = np.random.get_state()
    return [s[0], s[1].tolist(), int(s[2]), int(s[3]), float(s[4])]


def load_full_checkpoint(path: str) -> Dict[str, Any]:
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if obj.get("format") != "pytorch_r2d2_amd.full.v1":
        raise ValueError(f"{path} is not a full-state checkpoint")
    return obj


def restore_rng(obj: Dict[str, Any]) -> None:
    torch.set_rng_state(obj["torch_rng"])
    s = json.loads(obj["numpy_rng_json"])
    np.random.set_state((s[0], np.asarray(s[1], dtype=np.uint32), s[2], s[3], s[4]))
