"""Throughput of the drop-in trainer itself: MolCLR.train_step (molclr.py:107-128
loop body) over batches from the config's data module with the views built
on the device (DeviceViewLoader), i.e. exactly what ``MolCLR.train()`` runs
per step -- not bench.py's resident pre-built batches.

    python tools/trainer_bench.py [--config c2|c3|c5] [--aug node|subgraph|mix]
                                  [--data synthetic:<n> | file.txt | shard]
                                  [--epoch-steps 200] [--warmup 10] [--eager]

Runs ONE full epoch of the train loader (``--epoch-steps`` batches plus the
warm-up; the synthetic data set is sized to it, valid_size 0.05) through
MolCLR.train_step, and times every step after the first ``--warmup``.  The
HIP-graph step is the trainer's default (``hip_graph``); the line reports the
captures made during the warm-up and during the timed steps (a capacity-fit
lookup should make the latter ~0 after the first few batches).

Prints one JSON line: molecules/s, ms per step (wall over the timed steps,
and the median of per-step events), captures, where the views came from.
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
    ap.add_argument("--epoch-steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--eager", action="store_true", help="hip_graph: False")
    args = ap.parse_args()
    import torch

    from molclr_amd.molclr import MolCLR
    c = CFG[args.config]
    B = c["batch"]
    n_batches = args.epoch_steps + args.warmup
    # valid_size 0.05: the train split holds n_batches full batches
    data = args.data or f"synthetic:{int(B * n_batches / 0.95) + B}"
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
        "hip_graph": not args.eager,
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

    cs0 = trainer._graph_step(model, optimizer)
    if cs0 is not None and hasattr(train_loader, "on_epoch_plan"):
        train_loader.on_epoch_plan = cs0.prepare_sizes  # as MolCLR.train sets it
    it = iter(train_loader)
    steps_in_epoch = len(train_loader)
    for i in range(args.warmup):
        xi, xj = next(it)
        loss = trainer.train_step(model, optimizer, xi, xj, i)
    torch.cuda.synchronize()
    cs = getattr(trainer, "_captured", None)
    cap_warm = cs.captures if cs is not None else 0
    timed = steps_in_epoch - args.warmup
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(timed + 1)]
    cap_at = []
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(timed):
        xi, xj = next(it)
        loss = trainer.train_step(model, optimizer, xi, xj, args.warmup + i)
        marks[i + 1].record()
        if cs is not None:
            cap_at.append(cs.captures)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    trainer.check_inputs()
    step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(timed)]
    cap_timed = (cs.captures - cap_warm) if cs is not None else 0
    last_capture_step = None
    if cs is not None and cap_timed:
        last_capture_step = args.warmup + next(i for i, c in enumerate(cap_at) if c == cs.captures)
    print(json.dumps({
        "what": "MolCLR.train_step over one epoch of DeviceViewLoader batches (views built on "
                "the GPU), " + ("HIP-graph step" if cs is not None else "eager step"),
        "config": args.config, "aug": args.aug, "data": data, "batch": B,
        "epoch_steps": steps_in_epoch, "warmup_steps": args.warmup, "timed_steps": timed,
        "molecules_per_s": round(B * timed / wall, 1),
        "ms_per_step": round(wall / timed * 1e3, 3),
        "median_step_ms": round(statistics.median(step_ms), 3),
        "median_molecules_per_s": round(B / (statistics.median(step_ms) / 1e3), 1),
        "captures_warmup": cap_warm, "captures_timed": cap_timed,
        "last_capture_step": last_capture_step,
        "buckets": sorted(cs.buckets) if cs is not None else None,
        "store_build_s": round(t_store, 2), "final_loss": round(float(loss.item()), 5),
    }), flush=True)


if __name__ == "__main__":
    main()
