"""Phase timeline of the persistent fused step (kernels/mlp_persist.hip):
layer-1 block 0, chain block 0 and gradient block 0, steps 8..15 of one launch
(s_memrealtime, 100 MHz -> us).  Prints per-phase medians and writes JSON to
argv[1]; argv[2] = model (default 784-128-64-10)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

C = require_native()
L1 = ["fwd+publish", "dZ1 wait", "bwd+update"]
CH = ["partials flags wait", "partials load+H1, W wait+load", "fwd+softmax", "bwd+dZ1 publish",
      "rows publish"]
GB = ["rows wait+load", "dW/db MFMAs", "exchange+update", "publish"]


def decode(v, spec) -> dict:
    """Phase medians (us) from mlp_persist_stamps() of a stamped launch."""
    st = [[[v[(r * 8 + s) * 8 + p] for p in range(8)] for s in range(8)] for r in range(4)]
    out = {"model": str(spec), "layer1": {}, "chain": {}, "grad": {}, "step_us": None}
    med = lambda xs: round(statistics.median(xs), 3)  # noqa: E731
    for name, role, labels in (("layer1", 0, L1), ("chain", 1, CH), ("grad", 2, GB)):
        for k, lab in enumerate(labels):
            d = [(st[role][s][k + 1] - st[role][s][k]) / 100.0 for s in range(8)
                 if st[role][s][k + 1] and st[role][s][k]]
            out[name][lab] = med(d) if d else None
    out["step_us"] = med([(st[0][s + 1][0] - st[0][s][0]) / 100.0 for s in range(7)])
    # cross-role hand-offs: layer-1 publish -> chain has H1; chain dZ1 publish ->
    # layer-1 has dZ1; chain rows -> gradient block has them; gradient publish ->
    # chain has the next step's weights
    out["l1_publish_to_chain_h1_us"] = med([(st[1][s][2] - st[0][s][1]) / 100.0 for s in range(8)])
    out["chain_dz1_publish_to_l1_ready_us"] = med([(st[0][s][2] - st[1][s][4]) / 100.0 for s in range(8)])
    out["chain_rows_to_grad_ready_us"] = med([(st[2][s][1] - st[1][s][5]) / 100.0 for s in range(8)])
    out["grad_publish_to_chain_w_ready_us"] = med([(st[1][s + 1][1] - st[2][s][4]) / 100.0 for s in range(7)])
    out["chain_flag_wait_us"] = med([(st[1][s][1] - st[1][s][0]) / 100.0 for s in range(8)])
    if all(st[1][s][6] for s in range(8)):
        # Gram forms: chain step start -> Z1 poll begins (weights fetched first
        # for 2 layers) -> Z1 seen; layer-1 gk = 0 block: dZ1 ready -> Z1 = P + C
        # stored; Z1 stored (step s) -> chain sees it (step s+1)
        out["gram"] = {
            "chain_start_to_z1_poll_us": med([(st[1][s][6] - st[1][s][0]) / 100.0 for s in range(8)]),
            "chain_z1_poll_us": med([(st[1][s][1] - st[1][s][6]) / 100.0 for s in range(8)]),
            "l1_dz1_ready_to_z1_stored_us": med([(st[0][s][4] - st[0][s][2]) / 100.0 for s in range(8)]),
            "l1_z1_stored_to_step_end_us": med([(st[0][s][3] - st[0][s][4]) / 100.0 for s in range(8)]),
            "z1_stored_to_chain_seen_us": med([(st[1][s + 1][1] - st[0][s][4]) / 100.0 for s in range(7)]),
        }
        if all(st[0][s][6] for s in range(8)):
            # data-parallel Gram forms (merged poll): layer-1 block 0 (a gatherer)
            # before the poll -> every replica's dZ1 rows in LDS -> Z1 stored
            out["gram"]["l1_dz1_poll_us"] = med([(st[0][s][6] - st[0][s][2]) / 100.0 for s in range(8)])
            out["gram"]["l1_correction_publish_us"] = med([(st[0][s][4] - st[0][s][6]) / 100.0 for s in range(8)])
            out["gram"]["chain_dz1_publish_to_l1_rows_us"] = med(
                [(st[0][s][6] - st[1][s][4]) / 100.0 for s in range(8)])
            if all(st[0][s][5] and st[0][s][7] for s in range(8)):
                # the correction split: wave 0's MFMAs -> every wave's (barrier) -> Z1 stored
                out["gram"]["l1_corr_mfma_us"] = med([(st[0][s][5] - st[0][s][6]) / 100.0 for s in range(8)])
                out["gram"]["l1_corr_barrier_us"] = med([(st[0][s][7] - st[0][s][5]) / 100.0 for s in range(8)])
                out["gram"]["l1_corr_store_us"] = med([(st[0][s][4] - st[0][s][7]) / 100.0 for s in range(8)])
        elif all(st[0][s][5] for s in range(8)):
            # single replica: the correction block of column 0 (chains' XCD)
            out["gram"]["chain_dz1_publish_to_cb_seen_us"] = med(
                [(st[0][s][5] - st[1][s][4]) / 100.0 for s in range(8)])
            out["gram"]["cb_dz1_seen_to_z1_stored_us"] = med(
                [(st[0][s][4] - st[0][s][5]) / 100.0 for s in range(8)])
    if all(st[2][s][5] and st[2][s][6] and st[2][s][7] for s in range(8)):
        # data-parallel Gram forms: the gradient tile's exchange, split (tile 0, wave 0)
        out["grad_xchg"] = {
            "stage_us": med([(st[2][s][5] - st[2][s][2]) / 100.0 for s in range(8)]),
            "gather_us": med([(st[2][s][6] - st[2][s][5]) / 100.0 for s in range(8)]),
            "gathered_to_all_waves_us": med([(st[2][s][7] - st[2][s][6]) / 100.0 for s in range(8)]),
            "update_us": med([(st[2][s][3] - st[2][s][7]) / 100.0 for s in range(8)]),
        }
    gd = [[v[(3 * 8 + 2 + r) * 8 + p] for p in range(4)] for r in range(6)]
    if all(all(x) for x in gd):
        # tile 0 wave 0's px_tagged_gather, steps 8..13: entry -> loads issued ->
        # first round's data in -> sum done
        out["grad_gather"] = {
            "issue_us": med([(x[1] - x[0]) / 100.0 for x in gd]),
            "data_us": med([(x[2] - x[1]) / 100.0 for x in gd]),
            "rest_us": med([(x[3] - x[2]) / 100.0 for x in gd]),
        }
    out["upper_group_xcd_local"] = bool(v[(3 * 8 + 1) * 8 + 0])
    return out


if __name__ == "__main__":
    spec = MlpSpec.parse(sys.argv[2]) if len(sys.argv) > 2 else MlpSpec((784, 128, 64, 10))
    t = MlpTrainer(spec, synthetic_mnist(64 * 100, seed=1), batch=64, lr=0.01,
                   ctx=DistContext(device=torch.device("cuda", 0)))
    assert t.persistent
    t.train_steps(100)
    t.synchronize()
    # STAMP_FIRST=k: steps k .. k+7 of a driver-shaped launch (STAMP_STEPS, default
    # 20) instead of steps 8-15 of a 32-step one -- k = 0 shows a launch's ramp
    first = os.environ.get("STAMP_FIRST")
    if first is not None:
        C.mlp_persist_set_stamp_window(int(first))
        t.train_steps(int(os.environ.get("STAMP_STEPS", "20")))
    else:
        C.mlp_persist_set_stamping(True)
        t.train_steps(32)
    t.synchronize()
    C.mlp_persist_set_stamping(False)
    out = decode(C.mlp_persist_stamps(), spec)
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)
