"""Throughput of the drop-in trainer itself: MolCLR.train_step (molclr.py:107-128
loop body) over batches from the config's data module with the views built
on the device (DeviceViewLoader), i.e. exactly what ``MolCLR.train()`` runs
per step -- not bench.py's resident pre-built batches.

    python tools/trainer_bench.py [--config c2|c3|c5] [--aug node|subgraph|mix]
                                  [--data synthetic:8192 | file.txt | shard]
                                  [--steps 40] [--warmup 10]

Prints one JSON line: molecules/s, ms per step (median of per-step events and
wall over the timed steps), and where the views came from.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

CFG = {
    "c2": dict(model_type="gin", num_layer=5, emb_dim=300, batch=512, fp16=False, shape="uniform"),
    "c3": dict(model_type="gcn", num_layer=5, emb_dim=300, batch=512, fp16=False, shape="uniform"),
    "c5": dict(model_type="gin", num_layer=5, emb_dim=512, batch=1024, fp16=True, shape="pubchem"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CFG))
    ap.add_argument("--aug", default="node", choices=("node", "subgraph", "mix"))
    ap.add_argument("--data", default=None)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    args = ap.parse_args()
    import torch

    from molclr_amd.molclr import MolCLR
    c = CFG[args.config]
    B = c["batch"]
    data = args.data or f"synthetic:{B * 24}"
    config = {
        "batch_size": B, "warm_up": 10, "epochs": 100, "load_model": "None",
        "eval_every_n_epochs": 1, "save_every_n_epochs": 5, "log_every_n_steps": 50,
        "fp16_precision": c["fp16"], "init_lr": 0.0005, "weight_decay": "1e-5",
        "gpu": "cuda:0", "model_type": c["model_type"],
        "model": {"num_layer": c["num_layer"], "emb_dim": c["emb_dim"], "feat_dim": 512,
                  "drop_ratio": 0, "pool": "mean"},
        "aug": args.aug,
        "dataset": {"num_workers": 12, "valid_size": 0.05, "data_path": data},
        "loss": {"temperature": 0.1, "use_cosine_similarity": True},
        "log_root": "/tmp/molclr_trainer_bench",
    }
    if args.aug == "node":
        from molclr_amd.dataset import MoleculeDatasetWrapper
    elif args.aug == "subgraph":
        from molclr_amd.dataset_subgraph import MoleculeDatasetWrapper
    else:
        from molclr_amd.dataset_mix import MoleculeDatasetWrapper
    ds = MoleculeDatasetWrapper(B, shape=c["shape"], **config["dataset"])
    trainer = MolCLR(ds, config)
    t0 = time.perf_counter()
    train_loader, _ = ds.get_data_loaders()
    t_store = time.perf_counter() - t0
    torch.manual_seed(0)
    model = trainer.build_model()
    optimizer, _ = trainer.build_optimizer(model)

    def batches():
        while True:
            yield from train_loader

    it = batches()
    for i in range(args.warmup):
        xi, xj = next(it)
        loss = trainer.train_step(model, optimizer, xi, xj, i)
    torch.cuda.synchronize()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        xi, xj = next(it)
        loss = trainer.train_step(model, optimizer, xi, xj, args.warmup + i)
        marks[i + 1].record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    trainer.check_inputs()
    step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
    print(json.dumps({
        "what": "MolCLR.train_step on DeviceViewLoader batches (views built on the GPU)",
        "config": args.config, "aug": args.aug, "data": data, "batch": B,
        "molecules_per_s": round(B * args.steps / wall, 1),
        "ms_per_step": round(wall / args.steps * 1e3, 3),
        "median_step_ms": round(statistics.median(step_ms), 3),
        "store_build_s": round(t_store, 2), "final_loss": round(float(loss.item()), 5),
    }), flush=True)


if __name__ == "__main__":
    main()
