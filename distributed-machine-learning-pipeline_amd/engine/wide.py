"""Wide-MLP engine (BASELINE config 4: MLP 784-4096-4096-10, bf16 on MI355X).

Mixed precision: fp32 master weights, bf16 activations, fp32 accumulation,
fp32 gradients all-reduced across replicas.  Each fp32 master W is stored
SPLIT, losslessly: its bf16 high half (rounded half away from zero) IS the
bf16 copy the GEMMs read, in W's stored [out][in] layout, and an int16
remainder holds the rest of the bits (kernels/wgrad_sgd.hip hl_*).  The
update reads and writes 4 B per weight instead of fp32 W + a separate bf16
copy (10 B): 20 % fewer bytes in the HBM-bound weight-update kernel.  The
flat fp32 parameter vector (models/mlp.py layout) holds the biases; its
weight part is rebuilt from the split masters on demand (`params()`).  No transposed copy of anything:
the products that reduce over a strided dimension read their operand through
gfx950's transposing LDS read (ds_read_b64_tr_b16).

Per step, with L layers (every kernel hand-written for gfx950 MFMA):
  cast      X (fp32) -> bf16
  forward   H_{l+1} = relu(H_l . W_l^T + b_l)   kernels/gemm_skinny.hip NT (split-K,
            64x64 tiles, >= 256 workgroups) or gemm_rows64 for short K
  head      logits, softmax-CE, dZ_L and dZ_{L-1} = (dZ_L . W_{L-1}) * (H > 0)
            in one kernel (gemm_bf16.hip head_softmax_xent)
  dgrad     dZ_l = (dZ_{l+1} . W_l) * (H_l > 0)  gemm_skinny.hip NN (W untransposed)
  wgrad     W_l -= lr * dZ_{l+1}^T H_l, bf16 W_l refreshed, b_l step
            (kernels/wgrad_sgd.hip, straight from the row-major activations)
  input     one replica: the last dgrad leaves raw split-K slices and ONE
            launch (kernels/wide_input.hip) sums them into dZ_1, steps W_0 / b_0
            and computes the NEXT step's H_1 from the updated rows (so the step
            has no separate input-layer forward); bit-identical to the
            separate kernels
With several replicas, two gradient syncs:
  rccl / ring / torch   the wgrad kernel writes the gradient instead, and each
            layer's bucket is all-reduced + applied on a comm stream that
            overlaps the backward of the layers below (fp32, 4 B per weight:
            80 MB per step for 784-4096-4096-10);
  xact      activation exchange: every weight gradient of a 64-row batch is
            dZ_{l+1}^T H_l, so instead of the 80 MB of gradients the replicas
            all-gather the bf16 activations and activation gradients (H_l,
            dZ_l: 64 x 4096 x 2 B = 512 KB each, about 2 MB per replica per
            step) on the comm stream as each is produced, and every replica
            runs the fused weight-gradient + SGD launch over the whole global
            batch (M = 64 N rows, alpha = 1/N).  Identical inputs, identical
            kernel: the replicas stay bit-identical with no gradient all-reduce.
Reference hot loop replaced: client.go:112-202.
"""
from __future__ import annotations

import math
import os
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
                 gemm: str = "skinny", serial_sync: bool = False, xblk: Optional[bool] = None):
        from ..ops.native import require_native

        self.C = require_native()
        self.ctx = ctx or DistContext(device=torch.device("cuda", 0))
        if self.ctx.device.type != "cuda":
            raise ValueError("WideMlpTrainer runs on a GPU")
        if batch % 8:
            raise ValueError("batch must be a multiple of 8 (16 B bf16 rows)")
        if spec.dims[-1] > 64:
            raise ValueError("softmax kernel supports <= 64 classes")
        if any(x % 8 for x in spec.dims[:-1]):
            raise ValueError("input / hidden widths must be multiples of 8 (16 B bf16 rows)")
        if sync not in ("rccl", "ring", "torch", "xact"):
            raise ValueError("sync must be 'rccl', 'ring', 'torch' (gradient all-reduce) or 'xact' "
                             "(activation all-gather)")
        if gemm not in ("skinny", "rows64"):
            raise ValueError("gemm must be 'skinny' (split-K 64x64 tiles) or 'rows64' (full-K "
                             "64x16 tiles) for the forward products")
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
        # the training shard is resident in HBM: stage it in the compute dtype
        # once (bf16 rows padded to 16 columns) instead of casting every batch
        self.Xb = torch.zeros(self.nbatches * batch, _rup(spec.dims[0], 16), dtype=torch.bfloat16,
                              device=dev)
        self.C.cast_transpose(self.X, self.nbatches * batch, spec.dims[0], self.Xb, None)
        self._P = init_params(self.layout, seed, init).to(dev)
        self.G = torch.zeros_like(self._P)
        bf = dict(dtype=torch.bfloat16, device=dev)
        # bf16 W_l with rows padded to 16 (zeros: the dgrad reads a whole K tile of
        # rows), double-buffered by step parity: step s reads Wb[l][s % 2] (forward,
        # dgrad, head) while its weight-gradient kernel writes the updated copy into
        # Wb[l][(s + 1) % 2] -- so a replica's comm-stream updates never race the
        # dgrad chain that still reads the old weights.
        self.Wb = [[torch.zeros(self.pd[l + 1], self.pd[l], **bf) for _ in range(2)]
                   for l in range(L)]
        # the int16 remainders of the split fp32 masters (updated in place)
        self.Wlo = [torch.zeros(self.pd[l + 1], self.pd[l], dtype=torch.int16, device=dev)
                    for l in range(L)]
        self.H = [None] + [torch.zeros(batch, self.pd[l], **bf) for l in range(1, L)]
        self.dZ = [None] + [torch.zeros(batch, self.pd[l], **bf) for l in range(1, L + 1)]
        self.xact = self.ctx.is_distributed and sync == "xact"
        self.logits = torch.zeros(batch, d[L], dtype=torch.float32, device=dev)
        # per-row loss / correct / count accumulators (the head kernel's row_stats
        # form: no same-address atomics), summed by read_stats
        self.stats = torch.zeros(batch * 4, dtype=torch.float32, device=dev)
        self.views = self.layout.views(self._P)
        self.gviews = self.layout.views(self.G)
        self.fused_head = d[L] <= 16 and self.pd[L - 1] <= 4096
        # the last hidden layer's split-K GEMM hands its raw slices to the head,
        # which sums them in slice order as it loads H (bias + ReLU on load,
        # H written back for the weight update): no ticket / combine / epilogue
        # tail in that GEMM (HIPDSML_WIDE_HEAD_SLABS=0: the in-GEMM combine)
        self.head_slabs = (os.environ.get("HIPDSML_WIDE_HEAD_SLABS", "1") == "1" and self.fused_head
                           and L >= 2 and batch <= 64 and d[L - 1] % 64 == 0)
        # split-K plans of the skinny GEMMs: name -> (M, N, K, nn, S)
        self.plans: Dict[str, tuple] = {}
        for l in range(L):
            if l < L - 1:
                self._plan(f"f{l}", batch, d[l + 1], d[l], False)
            if l > 0 and not (self.fused_head and l == L - 1):
                self._plan(f"b{l}", batch, d[l], self.pd[l + 1], True)
        # split-K workspace shared by every skinny GEMM of the step: the slices'
        # partial tiles and an arrival ticket per tile (kernels/gemm_skinny.hip)
        sizes = [self.C.gemm_skinny_ws(M, N, K, 0) for (M, N, K, _, _) in self.plans.values()]
        self.Cp = torch.zeros(max([w for w, _ in sizes] + [16]), dtype=torch.float32, device=dev)
        self.tctr = torch.zeros(max([c for _, c in sizes] + [1]), dtype=torch.int32, device=dev)
        self.steps_done = 0
        # One hipGraph per epoch (every batch offset baked in): replaying it
        # removes the host launches per step.  With several replicas the
        # per-layer RCCL all-reduces and updates on the comm stream are
        # captured too (fork/join of the comm stream inside the capture); only
        # the torch.distributed fallback (sync='torch', e.g. gloo) stays eager.
        self.comm = None
        if self.ctx.is_distributed and (sync in ("rccl", "ring") or
                                        (sync == "xact" and self.ctx.backend == "nccl")):
            self.comm = make_native_comm(self.ctx)
        # collectives captured into the epoch graph only on request until a
        # multi-GPU run has validated it; eager otherwise
        capture_comm = os.environ.get("HIPDSML_CAPTURE_COLLECTIVES", "0") == "1"
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
        # serial_sync: each bucket's all-reduce + update on the compute stream (no
        # overlap) -- the reference the overlapped schedule must match bit for bit
        self.serial_sync = serial_sync
        self._comm_delay_cycles = 0  # test hook: stall the comm stream before each bucket
        if self.comm is not None and sync == "ring":
            # the in-house ring's reduce scratch, sized once for the largest bucket
            self.comm.reserve_ring(max(hi - lo for lo, hi in self._gspan), 4 << 20)
        # an epoch graph must start at an even step (the Wb parity it baked in)
        self.period = self.nbatches if self.nbatches % 2 == 0 else 2 * self.nbatches
        # xblk: the input-layer GEMM reads a k-blocked copy of the shard
        # ([K/32][rows][32] bf16): a 16-row MFMA fragment load is then 1 KiB
        # contiguous instead of 16 half cache lines (gemm_bf16.hip rows64 ABLK).
        # Same products, same order: bit-identical.
        if xblk is None:
            xblk = os.environ.get("HIPDSML_WIDE_XBLK", "1") == "1"
        self.Xblk = None
        if xblk and not self.xact and 512 <= d[0] <= 1024 and batch <= 64 \
                and (self.gemm == "rows64" or d[0] < 1024):
            nb = _rup(d[0], 32) // 32
            xp = torch.zeros(self.Xb.shape[0], nb * 32, **bf)
            xp[:, :d[0]] = self.Xb[:, :d[0]]
            self.Xblk = xp.view(-1, nb, 32).transpose(0, 1).contiguous()
            del xp
        if self.xact:
            self._init_xact(batch)
        # fused input layer (one replica): the last dgrad leaves raw split-K
        # slices, and ONE launch (kernels/wide_input.hip) sums them into dZ_1,
        # updates W_0 / b_0 and computes the NEXT step's H_1 with the updated
        # rows -- the input-layer forward launch and the dgrad's combine tail
        # leave the step.  Bit-identical to the separate kernels.  H_1 is
        # double-buffered by step parity (this step's H_1 is still read by the
        # update of W_1 while the next one is written); _carry is the step whose
        # H_1 is already in its buffer (None: run the forward first).
        self.fused_input = (os.environ.get("HIPDSML_WIDE_FUSED_INPUT", "1") == "1" and not self.ctx.is_distributed
                            and L >= 3 and batch == 64 and d[0] % 16 == 0 and d[0] <= 1024 and d[1] % 64 == 0
                            and self.head_slabs and self.plans["b1"][4] <= 8 and self.pd[0] == d[0])
        self._carry: Optional[int] = None
        self._input_beside = os.environ.get("HIPDSML_WIDE_INPUT_BESIDE", "1") == "1"
        if self.fused_input:
            self.H1buf = [self.H[1], torch.zeros_like(self.H[1])]
            # each batch's input rows twice more, in the fused launch's fragment
            # orders (static data, built once; 100 KB a batch each): XG for the
            # gradient ([K/16][2][16][32]: batch rows 32h + .. at 16 columns) and
            # XF for the forward (k-blocked [K/32][64][32]) -- every fragment load
            # is 1 KiB contiguous
            nb, k16, k32 = self.nbatches, _rup(d[0], 16), _rup(d[0], 32)
            xs = torch.zeros(nb, batch, k32, **bf)
            xs[:, :, :d[0]] = self.Xb[:nb * batch, :d[0]].view(nb, batch, d[0])
            self.XG = (xs[:, :, :k16].view(nb, 2, 32, k16 // 16, 16).permute(0, 3, 1, 4, 2).contiguous()
                       .view(nb, -1))
            self.XF = xs.view(nb, batch, k32 // 32, 32).permute(0, 2, 1, 3).contiguous().view(nb, -1)
            del xs
        self._refresh_bf16()

    def _init_xact(self, batch: int) -> None:
        """Gathered activation buffers: every H_l / dZ_l is a [N * batch, width]
        bf16 buffer whose rank-r rows are rank r's batch (this replica computes
        straight into its own slice; an in-place all-gather fills the rest).
        The inputs are exchanged once: all replicas' bf16 training shards,
        interleaved batch-major ([batch index][rank][row]), so each step's
        global input block is one contiguous [N * batch, 784] slice."""
        n, rk = self.ctx.world_size, self.ctx.rank
        lo, hi = self.ctx.all_reduce_scalars(float(self.nbatches), op="min")[0], \
            self.ctx.all_reduce_scalars(float(self.nbatches), op="max")[0]
        if lo != hi:
            raise ValueError("sync='xact' needs the same number of batches on every replica")
        bf = dict(dtype=torch.bfloat16, device=self.device)
        L = self.L
        self.Hall = [None] + [torch.zeros(n * batch, self.pd[l], **bf) for l in range(1, L)]
        self.dZall = [None] + [torch.zeros(n * batch, self.pd[l], **bf) for l in range(1, L + 1)]
        own = slice(rk * batch, (rk + 1) * batch)
        self.H = [None] + [self.Hall[l][own] for l in range(1, L)]
        self.dZ = [None] + [self.dZall[l][own] for l in range(1, L + 1)]
        rows = self.nbatches * batch
        full = torch.zeros(n * rows, self.Xb.shape[1], **bf)
        full[rk * rows:(rk + 1) * rows] = self.Xb[:rows]
        self._allgather_now(full)
        # [rank][batch][row] -> [batch][rank][row]
        self.Xall = (full.view(n, self.nbatches, batch, -1).transpose(0, 1).contiguous()
                     .view(self.nbatches * n * batch, -1))
        self.Xb = None  # the local rows are read from Xall

    def _allgather_now(self, full: torch.Tensor) -> None:
        """In-place all-gather of `full` (rank r's rows in part r) on the
        current stream: RCCL when the job has it, else torch.distributed with
        host staging (gloo rehearsals on one GPU)."""
        n = self.ctx.world_size
        if self.comm is not None:
            self.comm.allgather_(full)
            return
        import torch.distributed as dist

        host = full.cpu()
        parts = list(host.chunk(n))
        mine = parts[self.ctx.rank].clone()
        dist.all_gather(parts, mine)
        full.copy_(torch.cat(parts))

    def _gather(self, full: torch.Tensor) -> None:
        """All-gather one activation buffer on the comm stream once the compute
        stream has produced this replica's rows (in issue order on every rank)."""
        main = torch.cuda.current_stream(self.device)
        cs = main if self.serial_sync else self._cs
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            if self._comm_delay_cycles:
                torch.cuda._sleep(self._comm_delay_cycles)
            self._allgather_now(full)

    def _xb_rows(self, b: int) -> torch.Tensor:
        """This replica's bf16 input rows of batch b."""
        if self.xact:
            n, rk, Bt = self.ctx.world_size, self.ctx.rank, self.batch
            return self.Xall[(b * n + rk) * Bt:(b * n + rk + 1) * Bt]
        return self.Xb[b * self.batch:(b + 1) * self.batch]

    def _refresh_bf16(self) -> None:
        """Split masters (both hi copies + the remainders) from the fp32 W in P."""
        self._carry = None
        for l in range(self.L):
            W, _ = self.views[l]
            self.C.hilo_split(W, self.Wb[l][0], self.Wlo[l])
            self.Wb[l][1].copy_(self.Wb[l][0])

    def params(self) -> torch.Tensor:
        """The flat fp32 parameter vector, its weights rebuilt from the split
        masters (exact: the split is lossless)."""
        with torch.cuda.device(self.device):
            for l in range(self.L):
                W, _ = self.views[l]
                self.C.hilo_join(self.wb(l), self.Wlo[l], W)
        return self._P

    @property
    def P(self) -> torch.Tensor:
        return self.params()

    def wb(self, l: int) -> torch.Tensor:
        """The bf16 copy of W_l the next step reads."""
        return self.Wb[l][self.steps_done % 2]

    def _plan(self, name: str, M: int, N: int, K: int, nn: bool) -> None:
        self.plans[name] = (M, N, K, nn, self.C.gemm_skinny_splits(M, N, K, 0))

    def _slab_plan(self, l: int) -> int:
        """Slices of layer l's forward GEMM when the head combines them (0: the
        GEMM combines them itself)."""
        if not self.head_slabs or l != self.L - 2 or self.xact:
            return 0
        M, N, K, nn, S = self.plans[f"f{l}"]
        if self.gemm == "rows64" or K < 1024 or S not in (2, 4, 8):
            return 0
        return S

    def _last_hidden_and_head(self, cur_prev: torch.Tensor, W_head: torch.Tensor, rows: int, y: torch.Tensor,
                              logits, stats, dzp) -> None:
        """H_{L-1} = relu(H_{L-2} W^T + b) as raw split-K slices, then the head
        (kernels/head_row.h) sums them while it loads H, writes H_{L-1} back and
        runs the classifier + softmax-CE (+ dZ_{L-1})."""
        C, d, L = self.C, self.spec.dims, self.L
        l = L - 2
        M, N, K, nn, S = self.plans[f"f{l}"]
        _, b = self.views[l]
        _, bh = self.views[L - 1]
        C.gemm_skinny(self.H[l], cur_prev, rows, N, K, nn=False, ws=self.Cp, raw=True)
        C.head_softmax_xent(self.H[L - 1], W_head, bh, rows, self.pd[L - 1], d[L], y, 1.0 / rows, logits,
                            self.dZ[L], None, stats, dzp=dzp, row_stats=True, hs=self.Cp, hs_splits=S,
                            hs_bias=b, hs_relu=True)

    def _gemm(self, name: str, A: torch.Tensor, B: torch.Tensor, rows: int = 0, **epi) -> None:
        """One skinny GEMM with its epilogue fused (split-K combined in-kernel
        by the last slice of each tile to arrive); `rows` < batch for a short
        last batch (evaluation)."""
        M, N, K, nn, _ = self.plans[name]
        M = rows or M
        if not nn and (self.gemm == "rows64" or K < 1024):
            # short K: a 64 x 16 tile per block over the full K beats a split-K tail
            self.C.gemm_bf16_nt_fused(A, B, M, N, K, splits=0, **epi)
            return
        self.C.gemm_skinny(A, B, M, N, K, nn=nn, ws=self.Cp, ctr=self.tctr, **epi)

    # ----------------------------------------------------------------- step --
    def _x_operand(self, bi: int) -> torch.Tensor:
        """The input-layer forward's A operand for batch bi (k-blocked when built)."""
        r0 = bi * self.batch
        return self.Xblk[:, r0:r0 + self.batch] if self.Xblk is not None else self._xb_rows(bi)

    def _step(self) -> None:
        C, d, L, Bt = self.C, self.spec.dims, self.L, self.batch
        bi = self.steps_done % self.nbatches
        r0 = bi * Bt
        p = self.steps_done % 2
        cur = [self.Wb[l][p] for l in range(L)]       # this step's weights
        nxt = [self.Wb[l][1 - p] for l in range(L)]   # written by this step's updates
        self.H[0] = self._xb_rows(bi)  # this batch's bf16 rows (a view: no copy)
        slabs = self._slab_plan(L - 2)
        if self.fused_input:
            self.H[1] = self.H1buf[p]
        for l in range(L - 1):
            if slabs and l == L - 2:
                break  # the head combines this layer's GEMM (below)
            if l == 0 and self.fused_input and self._carry == self.steps_done:
                continue  # H_1 came with the previous step's input-layer launch
            _, b = self.views[l]
            A = self._x_operand(bi) if l == 0 else self.H[l]
            self._gemm(f"f{l}", A, cur[l], bias=b, relu=True, obf=self.H[l + 1])
            if self.xact:
                self._gather(self.Hall[l + 1])
        _, b = self.views[L - 1]
        if slabs:
            self._last_hidden_and_head(cur[L - 2], cur[L - 1], Bt, self.y[r0:r0 + Bt], self.logits, self.stats,
                                       self.dZ[L - 1])
        elif self.fused_head:  # classifier GEMM + softmax-CE in one kernel (one block per row),
            # plus the next activation gradient dZ_{L-1} from the W / H chunks it holds
            prev = L >= 2
            C.head_softmax_xent(self.H[L - 1], cur[L - 1], b, Bt, self.pd[L - 1], d[L],
                                self.y[r0:r0 + Bt], 1.0 / Bt, self.logits, self.dZ[L], None,
                                self.stats, dzp=self.dZ[L - 1] if prev else None, row_stats=True)
        else:
            C.gemm_bf16_nt_fused(self.H[L - 1], cur[L - 1], Bt, d[L], d[L - 1], bias=b,
                                 of32=self.logits, splits=0)
            C.softmax_xent(self.logits, self.y[r0:r0 + Bt], Bt, d[L], 1.0 / Bt, self.dZ[L],
                           None, self.stats)
        world = self.ctx.world_size
        fused_sgd = world == 1
        scale = self.lr / world
        main = torch.cuda.current_stream(self.device)
        if self.xact:
            self._gather(self.dZall[L])
            if self.fused_head and L >= 2:
                self._gather(self.dZall[L - 1])
            for l in range(L - 2 if self.fused_head else L - 1, 0, -1):
                self._gemm(f"b{l}", self.dZ[l + 1], cur[l], mask=self.H[l], obf=self.dZ[l])
                self._gather(self.dZall[l])
            main.wait_stream(self._cs)
            # every replica: the whole global batch's weight gradients (M = N x batch
            # rows, averaged by alpha = 1/N) with SGD fused, in one launch
            n, M = world, world * Bt
            Hall0 = self.Xall[bi * M:(bi + 1) * M]
            layers = []
            for l in range(L - 1, -1, -1):
                W, b = self.views[l]
                layers.append((self.dZall[l + 1], Hall0 if l == 0 else self.Hall[l], M, d[l + 1], d[l],
                               1.0 / n, self.lr, None, nxt[l], None, b, None, cur[l], self.Wlo[l]))
            for i in range(0, len(layers), 4):
                C.wgrad_sgd_multi(layers[i:i + 4])
            self.steps_done += 1
            return
        if fused_sgd and self.fused_input:
            # dgrads (the last one as raw slices), ONE launch for the layers above
            # the input layer, then the input layer's launch: dZ_1, W_0 / b_0 and
            # the next batch's H_1 (kernels/wide_input.hip)
            for l in range(L - 2, 0, -1):
                if l == 1:
                    M, N, K, _, S = self.plans["b1"]
                    C.gemm_skinny(self.dZ[2], cur[1], M, N, K, nn=True, ws=self.Cp, raw=True)
                else:
                    self._gemm(f"b{l}", self.dZ[l + 1], cur[l], mask=self.H[l], obf=self.dZ[l])
            layers = []
            for l in range(L - 1, 0, -1):
                W, b = self.views[l]
                layers.append((self.dZ[l + 1], self.H[l], Bt, d[l + 1], d[l], 1.0, scale, None, nxt[l],
                               None, b, None, cur[l], self.Wlo[l]))
            bn = (bi + 1) % self.nbatches
            _, b0 = self.views[0]
            args = (self.Cp, self.plans["b1"][4], self.H1buf[p], None, self.XG[bi], self.XF[bn], cur[0], self.Wlo[0],
                    nxt[0], b0, 1.0, scale, self.H1buf[1 - p], Bt, d[1], d[0])
            if self._input_beside and len(layers) <= 4:
                # the input layer's strips first in the update launch of the layers
                # above: their HBM phases overlap the tiles' weight stream
                C.wgrad_sgd_multi_in(layers, *args)
            else:
                for i in range(0, len(layers), 4):
                    C.wgrad_sgd_multi(layers[i:i + 4])
                C.wide_input_step(*args)
            self.steps_done += 1
            self._carry = self.steps_done
            return
        if fused_sgd:
            # every dgrad first (they read this step's bf16 weights), then ONE
            # launch updates every layer: W -= lr * dZ_{l+1}^T H_l, the next step's
            # bf16 copies, the biases (kernels/wgrad_sgd.hip, flattened tile grid)
            for l in range(L - 2 if self.fused_head else L - 1, 0, -1):
                self._gemm(f"b{l}", self.dZ[l + 1], cur[l], mask=self.H[l], obf=self.dZ[l])
            layers = []
            for l in range(L - 1, -1, -1):
                W, b = self.views[l]
                layers.append((self.dZ[l + 1], self.H[l], Bt, d[l + 1], d[l], 1.0, scale, None, nxt[l],
                               None, b, None, cur[l], self.Wlo[l]))
            for i in range(0, len(layers), 4):
                C.wgrad_sgd_multi(layers[i:i + 4])
            self.steps_done += 1
            return
        # several replicas, gradient all-reduce: per layer, the weight gradient,
        # then its bucket's all-reduce + SGD on the comm stream while the dgrad
        # of the layers below continues here
        for l in range(L - 1, -1, -1):
            gW, gb = self.gviews[l]
            if l > 0 and not (self.fused_head and l == L - 1):
                # activation gradient (reads this step's W_l copy, not the one being written)
                self._gemm(f"b{l}", self.dZ[l + 1], cur[l], mask=self.H[l], obf=self.dZ[l])
            C.wgrad_sgd(self.dZ[l + 1], self.H[l], Bt, d[l + 1], d[l], G=gW, bgrad=gb)
            self._sync_layer(l, scale, cur[l], nxt[l])
        # join: the next step's forward reads every updated layer (and overwrites
        # the activations the comm-stream updates read)
        main.wait_stream(self._cs)
        self.steps_done += 1

    def _sync_layer(self, l: int, scale: float, wb_cur: torch.Tensor, wb_next: torch.Tensor) -> None:
        """Per-layer gradient bucket: as soon as layer l's weight gradient is
        written, its all-reduce and its SGD + bf16 refresh run on the comm stream
        while the backward of layers < l continues on the compute stream (none of
        them reads W_l or the bf16 copy being written).  Buckets are whole
        layers, issued in the same order on every rank.  The refreshed bf16
        copy goes to the parity buffer the NEXT step reads."""
        C, d = self.C, self.spec.dims
        main = torch.cuda.current_stream(self.device)
        cs = main if self.serial_sync else self._cs
        cs.wait_stream(main)
        W, b = self.views[l]
        gW, gb = self.gviews[l]
        lo, hi = self._gspan[l]
        with torch.cuda.stream(cs):
            if self._comm_delay_cycles:
                torch.cuda._sleep(self._comm_delay_cycles)
            g = self.G[lo:hi]
            if self.comm is not None:
                (self.comm.ring_allreduce_(g, 0, 4 << 20) if self.sync == "ring"
                 else self.comm.allreduce_(g, 0))
            else:
                import torch.distributed as dist

                dist.all_reduce(g)
            C.hilo_sgd(wb_cur, self.Wlo[l], gW, scale, wb_next)
            C.sgd_update_(b, gb, scale)

    def _warm_comm(self) -> None:
        """Every bucket's collective once, eagerly, before any capture: RCCL
        sets up its channels / peer connections on the first call of a shape,
        and that host-side setup must not happen inside a stream capture.  G
        is scratch (rewritten by every step's weight-gradient GEMMs)."""
        if self.comm is None:
            return
        with torch.cuda.stream(self._cs):
            if self.xact:
                for buf in self.Hall[1:] + self.dZall[1:]:
                    self.comm.allgather_(buf)
                torch.cuda.synchronize(self.device)
                return
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
        # the graph's first step takes H_1 from the step before it (fused input layer)
        self._ensure_carry()
        carry = self._carry
        with torch.cuda.graph(g, stream=stream):
            for _ in range(self.period):
                self._step()
        self.steps_done = saved
        self._carry = carry
        self._graph = g

    def _ensure_carry(self) -> None:
        """Fused input layer: make this step's H_1 valid (the standalone forward
        of layer 0) when no previous step left it (first step, after evaluate /
        a checkpoint load)."""
        if not self.fused_input or self._carry == self.steps_done:
            return
        p, bi = self.steps_done % 2, self.steps_done % self.nbatches
        _, b = self.views[0]
        self._gemm("f0", self._x_operand(bi), self.Wb[0][p], bias=b, relu=True, obf=self.H1buf[p])
        self._carry = self.steps_done

    def train_steps(self, n: int) -> None:
        with torch.cuda.device(self.device):
            while n > 0:
                if (self.graph_enabled and self.steps_done % self.period == 0
                        and n >= self.period):
                    if self._graph is None:
                        self._capture_epoch()
                    self._ensure_carry()
                    self._graph.replay()
                    self._carry = self.steps_done + self.period
                    self.steps_done += self.period
                    n -= self.period
                else:
                    self._step()
                    n -= 1

    def synchronize(self) -> None:
        torch.cuda.synchronize(self.device)

    def read_stats(self, reset: bool = True, global_: bool = False) -> StepStats:
        self.synchronize()
        v = self.stats.view(-1, 4).sum(0).tolist()
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
        return {"spec": list(self.spec.dims), "params": self.params().detach().cpu().clone(),
                "velocity": torch.empty(0), "steps_done": self.steps_done, "lr": self.lr,
                "batch": self.batch}

    def load_state_dict(self, sd: Dict[str, object]) -> None:
        if list(sd["spec"]) != list(self.spec.dims):
            raise ValueError("checkpoint is for a different model")
        self.synchronize()
        self._P.copy_(sd["params"].to(self.device))
        self.steps_done = int(sd["steps_done"])
        self._carry = None
        self._refresh_bf16()  # the split masters from the fp32 weights
        self.synchronize()

    @torch.no_grad()
    def evaluate(self, ds: Dataset) -> Dict[str, float]:
        """Loss / accuracy of the current weights on the GPU kernels the step
        uses (bf16 GEMMs on the refreshed bf16 weight copies, fp32 accumulate,
        fused head + softmax-CE statistics), batch by batch."""
        C, d, L, Bt = self.C, self.spec.dims, self.L, self.batch
        X = ds.X.to(self.device, torch.float32).contiguous()
        y = ds.y.to(self.device, torch.int32).contiguous()
        n = X.shape[0]
        self._carry = None  # the activation buffers below are reused: H_1 is recomputed before the next step
        st = torch.zeros(Bt * 4, dtype=torch.float32, device=self.device)
        xb = torch.zeros(Bt, self.pd[0], dtype=torch.bfloat16, device=self.device)
        with torch.cuda.device(self.device):
            self.synchronize()
            for r0 in range(0, n, Bt):
                m = min(Bt, n - r0)
                C.cast_transpose(X[r0:r0 + m], m, d[0], xb, None)
                self.H[0] = xb
                slabs = self._slab_plan(L - 2)
                for l in range(L - 1):
                    if slabs and l == L - 2:
                        break
                    _, b = self.views[l]
                    self._gemm(f"f{l}", self.H[l], self.wb(l), rows=m, bias=b, relu=True,
                               obf=self.H[l + 1])
                _, b = self.views[L - 1]
                if slabs:
                    self._last_hidden_and_head(self.wb(L - 2), self.wb(L - 1), m, y[r0:r0 + m], None, st, None)
                elif self.fused_head:
                    C.head_softmax_xent(self.H[L - 1], self.wb(L - 1), b, m, self.pd[L - 1], d[L],
                                        y[r0:r0 + m], 1.0 / m, None, self.dZ[L], None, st,
                                        row_stats=True)
                else:
                    C.gemm_bf16_nt_fused(self.H[L - 1], self.wb(L - 1), m, d[L], d[L - 1], bias=b,
                                         of32=self.logits, splits=0)
                    C.softmax_xent(self.logits, y[r0:r0 + m], m, d[L], 1.0 / m, self.dZ[L], None, st)
            v = st.view(-1, 4).sum(0).tolist()
        return {"loss": v[0] / max(n, 1), "accuracy": 100.0 * v[1] / max(n, 1), "n": n}
