"""MLP model family: spec, flat parameter layout, initialisation, and the fp32
reference math used as the CPU backend and as the numerics oracle for the HIP
kernels.

Reference parity
----------------
* Model: the reference client codes 784-128-10 (``DSML/client/client.go:22-33``);
  its README/report claim 784-128-64-10 (``README.md:136-140``).  Any layer list
  is supported; the default is the BASELINE config 784-128-64-10.
* Init: U(-0.05, 0.05) for every weight and bias (``client.go:44-51``).
* Loss: softmax + CE with ``-log(p_y + 1e-10)`` averaged over the batch,
  ``dLogits = (p - y) / B`` (``client.go:143-165``); ReLU' masks ``z <= 0``
  (``client.go:104-110``); plain SGD ``w -= lr * g`` (``client.go:254-267``).

Layout
------
Weights use the PyTorch ``Linear`` convention ``W_l [out, in]`` so both GEMM
operands of the forward pass are K-contiguous (16 B vector loads on the GPU).
The reference stores ``W1[i*hidden + h]`` = ``[in, out]``; ``to_reference`` /
``from_reference`` convert the flat byte image used on the wire (``Memcpy`` of
the weights, ``client.go:204-218``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import numpy as np
import torch

MAX_LAYERS = 8
ROW_TILE = 16          # rows per workgroup of the fused row-chain kernel
LDS_BYTES = 160 * 1024  # gfx950 LDS per CU


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass(frozen=True)
class MlpSpec:
    dims: Tuple[int, ...] = (784, 128, 64, 10)

    def __post_init__(self):
        if len(self.dims) < 2 or len(self.dims) - 1 > MAX_LAYERS:
            raise ValueError(f"MLP needs 1..{MAX_LAYERS} layers, got dims={self.dims}")
        if any(d < 1 for d in self.dims):
            raise ValueError(f"bad dims {self.dims}")

    @property
    def nlayers(self) -> int:
        return len(self.dims) - 1

    @property
    def num_params(self) -> int:
        return sum(self.dims[i] * self.dims[i + 1] + self.dims[i + 1] for i in range(self.nlayers))

    @staticmethod
    def parse(s: str) -> "MlpSpec":
        return MlpSpec(tuple(int(x) for x in s.replace("x", "-").split("-") if x))

    def __str__(self) -> str:
        return "-".join(str(d) for d in self.dims)


@dataclass
class MlpLayout:
    """Flat fp32 parameter / workspace / LDS layout shared by Python and HIP."""

    spec: MlpSpec
    batch: int
    nbatches: int = 1
    w_off: List[int] = field(default_factory=list)
    b_off: List[int] = field(default_factory=list)
    act_off: List[int] = field(default_factory=list)
    dz_off: List[int] = field(default_factory=list)
    nparams: int = 0      # floats in the flat param buffer (incl. 64 B alignment padding)
    ws_floats: int = 0
    lds_act: List[int] = field(default_factory=list)
    lds_dz: List[int] = field(default_factory=list)
    lds_stride: List[int] = field(default_factory=list)
    lds_w: List[int] = field(default_factory=list)
    lds_b: List[int] = field(default_factory=list)
    lds_floats: int = 0
    w_in_lds: int = 1
    lab_off: int = 0

    def __post_init__(self):
        d = self.spec.dims
        L = self.spec.nlayers
        off = 0
        self.w_off, self.b_off = [], []
        for l in range(L):
            self.w_off.append(off)
            off = _rup(off + d[l + 1] * d[l], 16)
            self.b_off.append(off)
            off = _rup(off + d[l + 1], 16)
        self.nparams = off
        # workspace: H_l (l = 1..L-1), dZ_l (l = 1..L)
        self.act_off = [0] * (MAX_LAYERS + 1)
        self.dz_off = [0] * (MAX_LAYERS + 1)
        off = 0
        for l in range(1, L + 1):
            if l < L:
                self.act_off[l] = off
                off = _rup(off + self.batch * d[l], 16)
            self.dz_off[l] = off
            off = _rup(off + self.batch * d[l], 16)
        self.lab_off = off  # staged int32 labels of the current batch
        off = _rup(off + self.batch, 16)
        self.ws_floats = max(off, 16)
        # LDS of the row-chain kernel (floats, 16 B aligned)
        self.lds_act = [0] * (MAX_LAYERS + 1)
        self.lds_dz = [0] * (MAX_LAYERS + 1)
        self.lds_stride = [0] * (MAX_LAYERS + 1)
        self.lds_w = [0] * (MAX_LAYERS + 1)
        self.lds_b = [0] * (MAX_LAYERS + 1)
        off = 0
        for l in range(1, L + 1):
            st = _rup(d[l], 16) + 4
            self.lds_stride[l] = st
            self.lds_act[l] = off
            off += ROW_TILE * st
            self.lds_dz[l] = off
            off += ROW_TILE * st
        acts_only = off
        for l in range(2, L + 1):
            self.lds_w[l] = off
            off += d[l] * (d[l - 1] + 4)
            self.lds_b[l] = off
            off += _rup(d[l], 4)
        # Stage W_l (l >= 2) in LDS when it fits; otherwise the row chain reads
        # them from HBM/L2 and only the activation tiles live in LDS.
        if off * 4 <= LDS_BYTES:
            self.w_in_lds, self.lds_floats = 1, off
        else:
            self.w_in_lds, self.lds_floats = 0, acts_only

    # -- descriptor for the native runner (order: csrc/bindings.cpp) --------
    def desc_list(self) -> List[int]:
        A = MAX_LAYERS + 1
        dims = list(self.spec.dims) + [0] * (A - len(self.spec.dims))
        pad = lambda v, n: list(v) + [0] * (n - len(v))  # noqa: E731
        out = [self.spec.nlayers, self.batch, self.nbatches, self.w_in_lds]
        out += dims
        out += pad(self.lds_act, A) + pad(self.lds_dz, A) + pad(self.lds_stride, A)
        out += pad(self.lds_w, A) + pad(self.lds_b, A)
        out += [self.lds_floats]
        out += pad(self.w_off, MAX_LAYERS) + pad(self.b_off, MAX_LAYERS)
        out += pad(self.act_off, A) + pad(self.dz_off, A)
        out += [self.lab_off]
        return [int(x) for x in out]

    @property
    def fused_ok(self) -> bool:
        """True when the fused 3-kernel HIP step supports this model."""
        d = self.spec.dims
        return (self.lds_floats * 4 <= LDS_BYTES
                and all(x % 4 == 0 for x in d[:-1])
                and _rup(d[0], 16) // 16 <= 64)  # <= 8 splits of <= 128

    def with_batch(self, batch: int, nbatches: int = 1) -> "MlpLayout":
        return MlpLayout(self.spec, batch, nbatches)

    def slab_floats(self) -> int:
        kblocks = (self.spec.dims[0] + 15) // 16
        tiles = ((self.spec.dims[1] + 31) // 32) * ((self.batch + 31) // 32)
        want = (64 + tiles - 1) // tiles
        minsplit = (kblocks + 7) // 8
        nsplit = max(want, minsplit)
        if nsplit > 8 and minsplit <= 8:
            nsplit = 8
        nsplit = min(nsplit, kblocks)
        per = (kblocks + nsplit - 1) // nsplit
        nsplit = (kblocks + per - 1) // per
        return nsplit * self.batch * self.spec.dims[1]

    # -- views ---------------------------------------------------------------
    def views(self, flat: torch.Tensor) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        d = self.spec.dims
        out = []
        for l in range(self.spec.nlayers):
            W = flat[self.w_off[l]: self.w_off[l] + d[l + 1] * d[l]].view(d[l + 1], d[l])
            b = flat[self.b_off[l]: self.b_off[l] + d[l + 1]]
            out.append((W, b))
        return out

    # -- reference wire format ([in,out] weights, packed W1|b1|W2|b2...) -------
    def to_reference(self, flat: torch.Tensor) -> np.ndarray:
        parts = []
        for W, b in self.views(flat.detach().cpu().float()):
            parts.append(W.t().contiguous().reshape(-1).numpy())
            parts.append(b.numpy())
        return np.concatenate(parts).astype(np.float32)

    def from_reference(self, packed: np.ndarray, out: torch.Tensor | None = None) -> torch.Tensor:
        packed = np.asarray(packed, dtype=np.float32).reshape(-1)
        if packed.size != self.spec.num_params:
            raise ValueError(f"expected {self.spec.num_params} floats, got {packed.size}")
        flat = torch.zeros(self.nparams, dtype=torch.float32)
        d = self.spec.dims
        p = 0
        for l, (W, b) in enumerate(self.views(flat)):
            n = d[l] * d[l + 1]
            W.copy_(torch.from_numpy(packed[p:p + n].reshape(d[l], d[l + 1])).t())
            p += n
            b.copy_(torch.from_numpy(packed[p:p + d[l + 1]]))
            p += d[l + 1]
        if out is not None:
            out.copy_(flat.to(out.device))
            return out
        return flat


def init_params(layout: MlpLayout, seed: int = 0, scheme: str = "reference",
                device: str | torch.device = "cpu") -> torch.Tensor:
    """Flat fp32 params. ``reference``: U(-0.05, 0.05) for weights and biases
    (client.go:44-51); ``kaiming``: U(+-sqrt(6/fan_in)) weights, zero biases."""
    g = torch.Generator().manual_seed(seed)
    flat = torch.zeros(layout.nparams, dtype=torch.float32)
    for W, b in layout.views(flat):
        if scheme == "reference":
            W.copy_((torch.rand(W.shape, generator=g) - 0.5) * 0.1)
            b.copy_((torch.rand(b.shape, generator=g) - 0.5) * 0.1)
        elif scheme == "kaiming":
            bound = math.sqrt(6.0 / W.shape[1])
            W.copy_((torch.rand(W.shape, generator=g) * 2 - 1) * bound)
        else:
            raise ValueError(f"unknown init scheme {scheme}")
    return flat.to(device)


# ---------------------------------------------------------------------------
# fp32 reference math (CPU backend + oracle)
# ---------------------------------------------------------------------------
def forward_ref(layout: MlpLayout, flat: torch.Tensor, X: torch.Tensor):
    """Returns (logits, acts) with acts[0] = X and acts[l] = H_l (post-ReLU)."""
    acts = [X]
    h = X
    views = layout.views(flat)
    for l, (W, b) in enumerate(views):
        z = h @ W.t() + b
        if l < len(views) - 1:
            z = torch.relu(z)
            acts.append(z)
        h = z
    return h, acts


def loss_and_dlogits_ref(logits: torch.Tensor, y: torch.Tensor):
    """Softmax-CE exactly as client.go:143-165 (eps 1e-10, mean over batch)."""
    B = logits.shape[0]
    p = torch.softmax(logits, dim=1)
    py = p.gather(1, y.long().view(-1, 1)).squeeze(1)
    loss_sum = (-torch.log(py + 1e-10)).sum()
    onehot = torch.zeros_like(p).scatter_(1, y.long().view(-1, 1), 1.0)
    dlogits = (p - onehot) / B
    correct = (logits.argmax(dim=1) == y.long()).sum()
    return loss_sum, dlogits, correct


def grads_ref(layout: MlpLayout, flat: torch.Tensor, X: torch.Tensor, y: torch.Tensor):
    """Flat gradient (same layout as params) + (loss_sum, correct)."""
    logits, acts = forward_ref(layout, flat, X)
    loss_sum, dz, correct = loss_and_dlogits_ref(logits, y)
    g = torch.zeros_like(flat)
    gviews = layout.views(g)
    views = layout.views(flat)
    for l in range(layout.spec.nlayers - 1, -1, -1):
        gW, gb = gviews[l]
        gW.copy_(dz.t() @ acts[l])
        gb.copy_(dz.sum(0))
        if l > 0:
            W, _ = views[l]
            dz = (dz @ W) * (acts[l] > 0).to(dz.dtype)
    return g, loss_sum, correct
