"""Tensor-level ops: GPU tensors go to the hand-written HIP kernels (mandatory),
host tensors use the equivalent PyTorch reference math (for CPU-only tests and
the simulated device runtime).
"""
from __future__ import annotations

import torch

from .native import require_native

SUM, PROD, MIN, MAX = 0, 1, 2, 3
OP_NAMES = {"sum": SUM, "prod": PROD, "min": MIN, "max": MAX}


def _op_id(op) -> int:
    if isinstance(op, str):
        return OP_NAMES[op.lower()]
    return int(op)


def reduce_ref(a: torch.Tensor, b: torch.Tensor, op) -> torch.Tensor:
    """Reference elementwise reduction. u8 wraps like the reference's byte
    arithmetic (gpu_coordinator_server.go:542)."""
    op = _op_id(op)
    if a.dtype in (torch.bfloat16, torch.float16):
        af, bf = a.float(), b.float()
        out = _reduce_f(af, bf, op)
        return out.to(a.dtype)
    if a.dtype == torch.uint8:
        ai, bi = a.to(torch.int32), b.to(torch.int32)
        out = _reduce_f(ai, bi, op)
        return (out & 0xFF).to(torch.uint8)
    return _reduce_f(a, b, op)


def _reduce_f(a, b, op):
    if op == SUM:
        return a + b
    if op == PROD:
        return a * b
    if op == MIN:
        return torch.minimum(a, b)
    if op == MAX:
        return torch.maximum(a, b)
    raise ValueError(f"bad reduce op {op}")


def reduce_into(dst: torch.Tensor, a: torch.Tensor, b: torch.Tensor, op="sum") -> torch.Tensor:
    if dst.is_cuda:
        require_native().reduce_into(dst, a, b, _op_id(op))
    else:
        dst.copy_(reduce_ref(a, b, op))
    return dst


def reduce_(dst: torch.Tensor, src: torch.Tensor, op="sum") -> torch.Tensor:
    return reduce_into(dst, dst, src, op)


def sgd_update_(P: torch.Tensor, G: torch.Tensor, scale: float) -> torch.Tensor:
    if P.is_cuda:
        require_native().sgd_update_(P, G, float(scale))
    else:
        P.sub_(G, alpha=float(scale))
    return P


def sgd_momentum_(P, G, V, lr, momentum, weight_decay=0.0, gscale=1.0):
    if P.is_cuda:
        require_native().sgd_momentum_(P, G, V, float(lr), float(momentum), float(weight_decay),
                                       float(gscale))
    else:
        g = G * gscale + weight_decay * P
        V.mul_(momentum).add_(g)
        P.sub_(V, alpha=lr)
    return P


def u8_to_f32(src: torch.Tensor, scale: float = 1.0 / 255.0) -> torch.Tensor:
    """idx pixel bytes -> f32 * scale (client.go:307-310)."""
    dst = torch.empty(src.shape, dtype=torch.float32, device=src.device)
    if src.is_cuda:
        require_native().u8_to_f32(dst, src.contiguous(), float(scale))
    else:
        dst.copy_(src.float() * scale)
    return dst


def scale_(x: torch.Tensor, alpha: float) -> torch.Tensor:
    if x.is_cuda:
        require_native().scale_(x, float(alpha))
    else:
        x.mul_(alpha)
    return x
