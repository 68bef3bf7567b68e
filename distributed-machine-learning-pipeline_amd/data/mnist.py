"""MNIST data path: idx (gzip) readers compatible with the reference loader, and
a synthetic 28x28 generator for hardware runs (no network, no dataset on the
GPU box).

Reference: ``LoadMNISTImages`` / ``LoadMNISTLabels`` (``DSML/client/client.go:269-350``):
idx3 magic 2051 big-endian header, pixels / 255 as f32; idx1 magic 2049 labels
(one-hot in the reference; class indices here — the loss kernel consumes the
index directly).  Paths ``data/{train,t10k}-*-idx?-ubyte.gz`` (``client.go:545-548``).
"""
from __future__ import annotations

import gzip
import os
import struct
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

IMAGE_MAGIC = 2051
LABEL_MAGIC = 2049
REFERENCE_DATA_DIR = "/root/reference/DSML/data"
# The reference's own t10k files, shipped with the tests so the real-digit
# checks also run where the reference tree is absent (e.g. the GPU box).
FIXTURE_DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tests", "fixtures", "mnist")


def default_data_dir(split: str = "t10k") -> str:
    """The reference's data directory when present, else the test fixtures."""
    for d in (REFERENCE_DATA_DIR, FIXTURE_DATA_DIR):
        if os.path.exists(os.path.join(d, f"{split}-images-idx3-ubyte.gz")):
            return d
    return REFERENCE_DATA_DIR


def _open(path: str):
    with open(path, "rb") as f:
        head = f.read(2)
    return gzip.open(path, "rb") if head == b"\x1f\x8b" else open(path, "rb")


def load_idx_images(path: str, normalize: bool = True) -> np.ndarray:
    """[N, rows*cols] uint8 (or f32 / 255 when normalize)."""
    with _open(path) as f:
        magic, n, rows, cols = struct.unpack(">IIII", f.read(16))
        if magic != IMAGE_MAGIC:
            raise ValueError(f"{path}: invalid magic number {magic} (want {IMAGE_MAGIC})")
        buf = f.read(n * rows * cols)
    if len(buf) != n * rows * cols:
        raise ValueError(f"{path}: truncated image data")
    x = np.frombuffer(buf, dtype=np.uint8).reshape(n, rows * cols)
    return (x.astype(np.float32) / 255.0) if normalize else x


def load_idx_labels(path: str) -> np.ndarray:
    with _open(path) as f:
        magic, n = struct.unpack(">II", f.read(8))
        if magic != LABEL_MAGIC:
            raise ValueError(f"{path}: invalid magic number {magic} (want {LABEL_MAGIC})")
        buf = f.read(n)
    if len(buf) != n:
        raise ValueError(f"{path}: truncated label data")
    return np.frombuffer(buf, dtype=np.uint8).astype(np.int32)


def one_hot(labels: np.ndarray, n: int = 10) -> np.ndarray:
    out = np.zeros((labels.size, n), dtype=np.float32)
    out[np.arange(labels.size), labels] = 1.0
    return out


@dataclass
class Dataset:
    X: torch.Tensor   # [N, d0] float32 (row stride multiple of 4)
    y: torch.Tensor   # [N] int32
    name: str = "synthetic"

    def __len__(self) -> int:
        return int(self.X.shape[0])

    def to(self, device) -> "Dataset":
        return Dataset(self.X.to(device), self.y.to(device), self.name)

    def shard(self, rank: int, world: int) -> "Dataset":
        n = len(self) // world
        return Dataset(self.X[rank * n:(rank + 1) * n], self.y[rank * n:(rank + 1) * n],
                       f"{self.name}[{rank}/{world}]")


def synthetic_mnist(n: int, seed: int = 0, dim: int = 784, nclasses: int = 10,
                    noise: float = 0.35) -> Dataset:
    """Learnable synthetic 28x28 'digits': per-class smooth prototypes (shared
    across ranks: fixed prototype seed) plus per-sample noise, clipped to [0,1]."""
    proto_rng = np.random.default_rng(1234)
    side = int(round(dim ** 0.5))
    protos = proto_rng.random((nclasses, dim), dtype=np.float32)
    if side * side == dim:  # smooth the prototypes spatially (digit-like blobs)
        p = protos.reshape(nclasses, side, side)
        for _ in range(2):
            p = (p + np.roll(p, 1, 1) + np.roll(p, -1, 1) + np.roll(p, 1, 2) + np.roll(p, -1, 2)) / 5
        p = p.reshape(nclasses, dim)
        # binary strokes: each class lights up the pixels above its own median
        protos = (p > np.median(p, axis=1, keepdims=True)).astype(np.float32)
    rng = np.random.default_rng(seed)
    y = rng.integers(0, nclasses, size=n).astype(np.int32)
    X = protos[y] + noise * rng.standard_normal((n, dim), dtype=np.float32)
    np.clip(X, 0.0, 1.0, out=X)
    return Dataset(torch.from_numpy(X), torch.from_numpy(y), "synthetic")


def load_mnist(data_dir: Optional[str] = None, split: str = "t10k",
               limit: Optional[int] = None) -> Dataset:
    data_dir = data_dir or default_data_dir(split)
    img = os.path.join(data_dir, f"{split}-images-idx3-ubyte.gz")
    lab = os.path.join(data_dir, f"{split}-labels-idx1-ubyte.gz")
    X = load_idx_images(img)
    y = load_idx_labels(lab)
    if X.shape[0] != y.shape[0]:
        raise ValueError("image/label count mismatch")
    if limit:
        X, y = X[:limit], y[:limit]
    return Dataset(torch.from_numpy(np.ascontiguousarray(X)), torch.from_numpy(y), f"mnist-{split}")


def mnist_available(data_dir: Optional[str] = None, split: str = "t10k") -> bool:
    data_dir = data_dir or default_data_dir(split)
    return os.path.exists(os.path.join(data_dir, f"{split}-images-idx3-ubyte.gz"))


def train_test_split(ds: Dataset, test_fraction: float = 0.2) -> Tuple[Dataset, Dataset]:
    n = len(ds)
    nt = int(n * (1 - test_fraction))
    return (Dataset(ds.X[:nt], ds.y[:nt], ds.name + "-train"),
            Dataset(ds.X[nt:], ds.y[nt:], ds.name + "-test"))
