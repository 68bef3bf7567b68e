"""Wide-MLP engine (BASELINE config 4: MLP 784-4096-4096-10, bf16 on MI355X).

Mixed precision: fp32 master weights (flat, same layout as models/mlp.py),
bf16 copies of W and W^T for the MFMA GEMMs (refreshed by the fused
update+cast kernel), bf16 activations (+ transposed copies for the weight
gradients), fp32 accumulation, fp32 gradients all-reduced across replicas.

Every product is a bf16 "NT" GEMM on v_mfma_f32_16x16x32_bf16
(kernels/gemm_bf16.hip), split-K for the skinny (M = batch) GEMMs so a step
fills the 256 CUs; the epilogue (bias / ReLU / ReLU'-mask / casts / transposed
copy) runs inside the GEMM, on the last K split of each tile to arrive.  The
weight-gradient GEMMs carry the SGD update (fp32 master W and the bf16 W / W^T
copies, vectorised through LDS) and the bias step (row sums of dZ^T) when there
is one replica.  Per step, with L layers: 1 input cast, L forward GEMMs,
softmax-CE, 2L-1 backward GEMMs (+ with several replicas, one all-reduce and
one update per layer, bucketed by layer on a comm stream that overlaps the
backward of the layers below).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from ..data.mnist import Dataset
from ..models.mlp import MlpLayout, MlpSpec, init_params
from ..parallel.dist import DistContext, make_native_comm
from .trainer import StepStats


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class WideMlpTrainer:
    def __init__(self, spec: MlpSpec, data: Dataset, batch: int = 64, lr: float = 0.01, *,
                 ctx: Optional[DistContext] = None, seed: int = 0, init: str = "kaiming",
                 sync: str = "rccl", target_wgs: int = 256, graph: bool = True,
                 gemm: str = "rows64"):
        from ..ops.native import require_native

        self.C = require_native()
        self.ctx = ctx or DistContext(device=torch.device("cuda", 0))
        if self.ctx.device.type != "cuda":
            raise ValueError("WideMlpTrainer runs on a GPU")
        if batch % 8:
            raise ValueError("batch must be a multiple of 8 (16 B bf16 rows)")
        if spec.dims[-1] > 64:
            raise ValueError("softmax kernel supports <= 64 classes")
        if gemm not in ("rows64", "splitk"):
            raise ValueError("gemm must be 'rows64' (full-K batch-row kernel) or 'splitk'")
        self.spec, self.batch, self.lr, self.sync, self.gemm = spec, batch, lr, sync, gemm
        self.device = dev = self.ctx.device
        self.target_wgs = target_wgs
        d = spec.dims
        L = spec.nlayers
        self.L = L
        self.pd = [_rup(x, 16) for x in d]
        self.layout = MlpLayout(spec, batch, 1)
        self.X = data.X.to(dev, torch.float32).contiguous()
        self.y = data.y.to(dev, torch.int32).contiguous()
        self.nbatches = len(data) // batch
        self.P = init_params(self.layout, seed, init).to(dev)
        self.G = torch.zeros_like(self.P)
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.Wb = [torch.zeros(d[l + 1], self.pd[l], **bf) for l in range(L)]
        self.WbT = [torch.zeros(self.pd[l], self.pd[l + 1], **bf) for l in range(L)]
        self.H = [torch.zeros(batch, self.pd[l], **bf) for l in range(L)]
        self.HT = [torch.zeros(self.pd[l], batch, **bf) for l in range(L)]
        self.dZ = [None] + [torch.zeros(batch, self.pd[l], **bf) for l in range(1, L + 1)]
        self.dZT = [None] + [torch.zeros(self.pd[l], batch, **bf) for l in range(1, L + 1)]
        self.logits = torch.zeros(batch, d[L], dtype=torch.float32, device=dev)
        self.stats = torch.zeros(4, dtype=torch.float32, device=dev)
        self.views = self.layout.views(self.P)
        self.gviews = self.layout.views(self.G)
        # split-K plans of the batch-row GEMMs: name -> (M, N, K, splits); the
        # weight-gradient GEMMs (K = batch) run unsplit with the SGD epilogue
        self.plans: Dict[str, tuple] = {}
        ws = 0
        for l in range(L):
            ws = max(ws, self._plan(f"f{l}", batch, d[l + 1], self.pd[l]))
            if l > 0:
                ws = max(ws, self._plan(f"b{l}", batch, d[l], self.pd[l + 1]))
        self.Cp = torch.zeros(ws if gemm == "splitk" else 16, dtype=torch.float32, device=dev)
        # split-K arrival counters (one per 64x64 tile; every GEMM leaves them 0)
        tiles = max(math.ceil(M / 64) * math.ceil(N / 64) for (M, N, _, _) in self.plans.values())
        self.tctr = torch.zeros(tiles, dtype=torch.int32, device=dev)
        self.steps_done = 0
        # One hipGraph per epoch (every batch offset baked in): replaying it
        # removes the ~25 host launches per step.  With several replicas the
        # per-layer RCCL all-reduces and updates on the comm stream are
        # captured too (fork/join of the comm stream inside the capture); only
        # the torch.distributed fallback (sync='torch', e.g. gloo) stays eager.
        import os

        self.comm = None
        if self.ctx.is_distributed and sync in ("rccl", "ring"):
            self.comm = make_native_comm(self.ctx)
        capture_comm = os.environ.get("HIPDSML_CAPTURE_COLLECTIVES", "1") != "0"
        self.graph_enabled = graph and (not self.ctx.is_distributed or
                                        (self.comm is not None and capture_comm))
        self._graph = None
        # per-layer gradient buckets (W_l and b_l plus any padding between them) and
        # the stream their all-reduce + SGD run on, overlapped with the backward
        lay = self.layout
        self._gspan = [(min(lay.w_off[l], lay.b_off[l]),
                        max(lay.w_off[l] + d[l + 1] * d[l], lay.b_off[l] + d[l + 1]))
                       for l in range(L)]
        self._cs = torch.cuda.Stream(dev) if self.ctx.is_distributed else None
        for l in range(L):  # bf16 copies of the initial weights
            W, _ = self.views[l]
            self.C.sgd_cast(W, None, d[l + 1], d[l], 0.0, self.Wb[l], self.WbT[l])

    def _plan(self, name: str, M: int, N: int, K: int) -> int:
        tiles = math.ceil(M / 64) * math.ceil(N / 64)
        # ~one workgroup per CU, <= 4 K splits: the last split of a tile reads
        # the other slabs in one batch (per-CU bytes, not HBM, bound these GEMMs)
        splits = max(1, min(math.ceil(self.target_wgs / tiles), max(1, K // 128), 4))
        S = self.C.gemm_num_splits(K, splits)
        self.plans[name] = (M, N, K, splits)
        return S * tiles * 4096  # slabs: one 64x64 fp32 tile per split

    def _gemm(self, name: str, A: torch.Tensor, B: torch.Tensor, **epi) -> int:
        """One GEMM with its epilogue fused (split-K reduced in-kernel by the
        last split of each tile)."""
        M, N, K, splits = self.plans[name]
        if self.gemm == "rows64":  # full K per block, no slabs
            return self.C.gemm_bf16_nt_fused(A, B, M, N, K, splits=0, **epi)
        return self.C.gemm_bf16_nt_fused(A, B, M, N, K, splits=splits, ws=self.Cp, ctr=self.tctr,
                                         **epi)

    # ----------------------------------------------------------------- step --
    def _step(self) -> None:
        C, d, L, Bt = self.C, self.spec.dims, self.L, self.batch
        r0 = (self.steps_done % self.nbatches) * Bt
        C.cast_transpose(self.X[r0:r0 + Bt], Bt, d[0], self.H[0], self.HT[0])
        fused_head = d[L] <= 16 and self.pd[L - 1] <= 4096 and self.gemm == "rows64"
        for l in range(L - 1 if fused_head else L):
            _, b = self.views[l]
            if l < L - 1:
                self._gemm(f"f{l}", self.H[l], self.Wb[l], bias=b, relu=True, obf=self.H[l + 1],
                           obfT=self.HT[l + 1])
            else:
                self._gemm(f"f{l}", self.H[l], self.Wb[l], bias=b, of32=self.logits)
        if fused_head:  # classifier GEMM + softmax-CE in one kernel (one block per row),
            # plus the next activation gradient dZ_{L-1} from the W / H chunks it holds
            _, b = self.views[L - 1]
            prev = L >= 2
            C.head_softmax_xent(self.H[L - 1], self.Wb[L - 1], b, Bt, self.pd[L - 1], d[L],
                                self.y[r0:r0 + Bt], 1.0 / Bt, self.logits, self.dZ[L], self.dZT[L],
                                self.stats, dzp=self.dZ[L - 1] if prev else None,
                                dzpT=self.dZT[L - 1] if prev else None)
        else:
            C.softmax_xent(self.logits, self.y[r0:r0 + Bt], Bt, d[L], 1.0 / Bt, self.dZ[L],
                           self.dZT[L], self.stats)
        world = self.ctx.world_size
        fused_sgd = world == 1
        scale = self.lr / world
        for l in range(L - 1, -1, -1):
            W, b = self.views[l]
            gW, gb = self.gviews[l]
            if l > 0 and not (fused_head and l == L - 1):
                # activation gradient first: it needs the pre-update W_l^T
                self._gemm(f"b{l}", self.dZ[l + 1], self.WbT[l], mask=self.H[l], obf=self.dZ[l],
                           obfT=self.dZT[l])
            if fused_sgd:
                # dW_l = dZ^T H_l with SGD fused in the GEMM epilogue: W -= lr*dW, the bf16
                # W / W^T copies refreshed, and the bias step from the row sums of dZ^T.
                C.gemm_bf16_nt_fused(self.dZT[l + 1], self.HT[l], d[l + 1], d[l], Bt, sgdW=W,
                                     lr=scale, obf=self.Wb[l], obfT=self.WbT[l], bsgd=b)
            else:
                C.gemm_bf16_nt_fused(self.dZT[l + 1], self.HT[l], d[l + 1], d[l], Bt, of32=gW,
                                     bgrad=gb)
                self._sync_layer(l, scale)
        if not fused_sgd:
            # the next step's forward reads every updated layer
            torch.cuda.current_stream(self.device).wait_stream(self._cs)
        self.steps_done += 1

    def _sync_layer(self, l: int, scale: float) -> None:
        """Per-layer gradient bucket: as soon as layer l's weight gradient is
        written, its all-reduce and its SGD + bf16 refresh run on the comm stream
        while the backward of layers < l continues on the compute stream (none of
        them reads W_l or its bf16 copies).  Buckets are whole layers, issued in
        the same order on every rank."""
        C, d = self.C, self.spec.dims
        main = torch.cuda.current_stream(self.device)
        self._cs.wait_stream(main)
        W, b = self.views[l]
        gW, gb = self.gviews[l]
        lo, hi = self._gspan[l]
        with torch.cuda.stream(self._cs):
            g = self.G[lo:hi]
            if self.comm is not None:
                (self.comm.ring_allreduce_(g, 0, 4 << 20) if self.sync == "ring"
                 else self.comm.allreduce_(g, 0))
            else:
                import torch.distributed as dist

                dist.all_reduce(g)
            C.sgd_cast(W, gW, d[l + 1], d[l], scale, self.Wb[l], self.WbT[l])
            C.sgd_update_(b, gb, scale)

    def _warm_comm(self) -> None:
        """Every bucket's collective once, eagerly, before any capture: RCCL
        sets up its channels / peer connections on the first call of a shape,
        and that host-side setup must not happen inside a stream capture.  G
        is scratch (rewritten by every step's weight-gradient GEMMs)."""
        if self.comm is None:
            return
        with torch.cuda.stream(self._cs):
            for lo, hi in self._gspan:
                g = self.G[lo:hi]
                (self.comm.ring_allreduce_(g, 0, 4 << 20) if self.sync == "ring"
                 else self.comm.allreduce_(g, 0))
        torch.cuda.synchronize(self.device)

    def _capture_epoch(self) -> None:
        self._warm_comm()
        torch.cuda.synchronize(self.device)
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        saved = self.steps_done
        with torch.cuda.graph(g, stream=stream):
            for _ in range(self.nbatches):
                self._step()
        self.steps_done = saved
        self._graph = g

    def train_steps(self, n: int) -> None:
        with torch.cuda.device(self.device):
            while n > 0:
                if (self.graph_enabled and self.steps_done % self.nbatches == 0
                        and n >= self.nbatches):
                    if self._graph is None:
                        self._capture_epoch()
                    self._graph.replay()
                    self.steps_done += self.nbatches
                    n -= self.nbatches
                else:
                    self._step()
                    n -= 1

    def synchronize(self) -> None:
        torch.cuda.synchronize(self.device)

    def read_stats(self, reset: bool = True, global_: bool = False) -> StepStats:
        self.synchronize()
        v = self.stats.tolist()
        if reset:
            self.stats.zero_()
        s = StepStats(v[0], v[1], v[2])
        if global_ and self.ctx.is_distributed:
            s = StepStats(*self.ctx.all_reduce_scalars(s.loss_sum, s.correct, s.count))
        return s

    def grads_for_test(self) -> torch.Tensor:
        return self.G

    def state_dict(self) -> Dict[str, object]:
        self.synchronize()
        return {"spec": list(self.spec.dims), "params": self.P.detach().cpu().clone(),
                "velocity": torch.empty(0), "steps_done": self.steps_done, "lr": self.lr,
                "batch": self.batch}

    def load_state_dict(self, sd: Dict[str, object]) -> None:
        if list(sd["spec"]) != list(self.spec.dims):
            raise ValueError("checkpoint is for a different model")
        self.synchronize()
        self.P.copy_(sd["params"].to(self.device))
        self.steps_done = int(sd["steps_done"])
        d = self.spec.dims
        for l in range(self.L):  # refresh the bf16 GEMM copies from the fp32 masters
            W, _ = self.views[l]
            self.C.sgd_cast(W, None, d[l + 1], d[l], 0.0, self.Wb[l], self.WbT[l])
        self.synchronize()

    @torch.no_grad()
    def evaluate(self, ds: Dataset) -> Dict[str, float]:
        """fp32 evaluation of the master weights (torch ops on the GPU)."""
        from ..models.mlp import forward_ref

        X = ds.X.to(self.device, torch.float32)
        y = ds.y.to(self.device).long()
        self.synchronize()
        logits, _ = forward_ref(self.layout, self.P, X)
        p = torch.softmax(logits, 1)
        loss = (-torch.log(p.gather(1, y.view(-1, 1)).squeeze(1) + 1e-10)).sum().item()
        correct = (logits.argmax(1) == y).sum().item()
        n = X.shape[0]
        return {"loss": loss / max(n, 1), "accuracy": 100.0 * correct / max(n, 1), "n": n}

