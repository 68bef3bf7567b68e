"""Checkpoint / resume.

The reference keeps the weights only in client RAM and has no checkpointing
(grep ``checkpoint|save|resume`` = 0).  A checkpoint here is the
flat fp32 parameter buffer (plus momentum) and the step counter — everything a
replica needs, since all DP replicas hold identical state.  Rank 0 writes;
every rank reads.

Optional keys of a single-replica persistent-step trainer
(engine/trainer.py state_dict): ``persist_carry``, the hand-off buffer with
the next step's layer-1 partials and correction (int64[kTotalG], about 0.95 MB,
twice the 437 KB of parameters), so a resume is bit-identical to an
uninterrupted run; and ``persist_meta`` (batch, nbatches, a Gram-table
fingerprint): a carry whose meta does not match the resuming trainer is
dropped and the first resumed step's Z1 is recomputed instead.

Format: a ``torch.save`` dict of tensors and plain scalars, written atomically
(temporary file + ``os.replace``) as ``<dir>/ckpt_<step>.pt``, and loaded
with ``torch.load(weights_only=True)`` so nothing in the file is executed.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Any, Dict, List, Optional

import torch

_PAT = re.compile(r"ckpt_(\d+)\.pt$")


def checkpoint_path(directory: str, step: int) -> str:
    return os.path.join(directory, f"ckpt_{step:09d}.pt")


def list_checkpoints(directory: str) -> List[str]:
    paths = [p for p in glob.glob(os.path.join(directory, "ckpt_*.pt")) if _PAT.search(p)]
    return sorted(paths, key=lambda p: int(_PAT.search(p).group(1)))


def latest_checkpoint(directory: str) -> Optional[str]:
    cps = list_checkpoints(directory) if directory and os.path.isdir(directory) else []
    return cps[-1] if cps else None


def save_state(state: Dict[str, Any], path: str) -> str:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_state(path: str) -> Dict[str, Any]:
    return torch.load(path, map_location="cpu", weights_only=True)


def save_checkpoint(trainer, directory: str, keep: int = 2, extra: Optional[Dict[str, Any]] = None,
                    rank: int = 0) -> Optional[str]:
    """Write ``trainer.state_dict()`` (rank 0 only) and prune to the newest `keep`."""
    state = trainer.state_dict()
    if rank != 0:
        return None
    if extra:
        state = {**state, "extra": dict(extra)}
    path = save_state(state, checkpoint_path(directory, int(state["steps_done"])))
    if keep > 0:
        for old in list_checkpoints(directory)[:-keep]:
            try:
                os.remove(old)
            except FileNotFoundError:
                pass
    return path


def resume(trainer, path_or_dir: str) -> Optional[Dict[str, Any]]:
    """Load a checkpoint file, or the newest one in a directory.  Returns the
    loaded state (None when the directory has no checkpoint yet)."""
    path = path_or_dir
    if os.path.isdir(path_or_dir):
        path = latest_checkpoint(path_or_dir)
        if path is None:
            return None
    state = load_state(path)
    trainer.load_state_dict(state)
    return state
