#!/usr/bin/env python3
"""Real-digit accuracy check: train on the reference's t10k digits (first 8,000)
and test on the held-out 2,000, with the reference's hyper-parameters (batch 64,
SGD lr 0.01, U(-0.05, 0.05) init; client.go:21-51) for the reference's number
of SGD steps (10 epochs x 937 batches ~= 75 epochs x 125 batches here).  Runs the
native HIP step on a GPU and the fp32 torch reference math on the CPU; prints
one JSON line.  The reference's own figure (92.89 %, README.md:204) comes from
the 60k train split, which the reference tree does not ship."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(dims, device, epochs: int):
    import torch

    from hipdsml.data.mnist import load_mnist, train_test_split
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel.dist import DistContext

    tr_ds, te_ds = train_test_split(load_mnist(split="t10k"), 0.2)
    t = MlpTrainer(MlpSpec(dims), tr_ds, batch=64, lr=0.01, ctx=DistContext(device=device), seed=0,
                   graph_steps=125 if device.type == "cuda" else 0)
    t0 = time.perf_counter()
    t.train_steps(t.nbatches * epochs)
    t.synchronize()
    wall = time.perf_counter() - t0
    ev = t.evaluate(te_ds)
    return {"model": "-".join(map(str, dims)), "device": device.type, "steps": t.nbatches * epochs,
            "test_accuracy": round(ev["accuracy"], 2), "test_loss": round(ev["loss"], 4),
            "train_s": round(wall, 3)}


def main() -> int:
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=75)
    ap.add_argument("--cpu", action="store_true", help="also run the fp32 torch reference on the CPU")
    a = ap.parse_args()
    out = []
    for dims in [(784, 128, 64, 10), (784, 128, 10)]:
        if torch.cuda.is_available():
            out.append(run(dims, torch.device("cuda", 0), a.epochs))
        if a.cpu or not torch.cuda.is_available():
            out.append(run(dims, torch.device("cpu"), a.epochs))
    print(json.dumps({"data": "reference t10k digits: train [0, 8000), test [8000, 10000)",
                      "batch": 64, "lr": 0.01, "runs": out}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
