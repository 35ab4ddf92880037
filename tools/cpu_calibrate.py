"""Calibrate the CPU baseline: time the oracle's reference
step (oracle/reference_cpu.py: PyG-semantics index_select / index_add_,
per-layer add_self_loops, materialised edge embeddings, the broadcast-cosine
NT-Xent of utils/nt_xent.py:40-45) at c1 / c2 / c3 on this host, 1 warm-up +
median of N steps, with the thread count given, and compare with the survey's
timings of the reference's own modules on the 8-core build container
(c1 ~57 ms, c2 3.8-4.2 s, c3 2.9-3.6 s per step).

    python tools/cpu_calibrate.py [threads] [steps]

Prints one JSON line per config (ms per step, the survey band, the ratio).
Also times the NT-Xent alone (the survey: fwd ~320-390 ms, bwd ~2.3-2.8 s at
B = 512, C = 256) to attribute any gap.
"""
from __future__ import annotations

import json
import os
import platform
import statistics
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from oracle.reference_cpu import RefGCN, RefGINet, RefNTXentLoss, ref_train_step  # noqa: E402

CFG = {"c1": ("gin", 3, 128, 64, (52.0, 62.0)), "c2": ("gin", 5, 300, 512, (3800.0, 4200.0)),
       "c3": ("gcn", 5, 300, 512, (2900.0, 3600.0))}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def time_step(kind, L, D, B, steps):
    torch.manual_seed(0)
    model = (RefGINet if kind == "gin" else RefGCN)(L, D, 512)
    crit = RefNTXentLoss("cpu", B, 0.1, True)
    opt = torch.optim.Adam(model.parameters(), 5e-4, weight_decay=1e-5)
    batches = SyntheticPairBatches(B, seed=0).take(2)
    ts = []
    for i in range(steps + 1):
        xi, xj = batches[i % 2]
        t0 = time.perf_counter()
        ref_train_step(model, crit, opt, xi, xj)
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts[1:]) * 1e3


def time_ntxent(B=512, C=256, reps=3):
    crit = RefNTXentLoss("cpu", B, 0.1, True)
    f, b = [], []
    for _ in range(reps + 1):
        zi = torch.nn.functional.normalize(torch.randn(B, C), dim=1).requires_grad_(True)
        zj = torch.nn.functional.normalize(torch.randn(B, C), dim=1).requires_grad_(True)
        t0 = time.perf_counter()
        loss = crit(zi, zj)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        f.append(t1 - t0)
        b.append(t2 - t1)
    return statistics.median(f[1:]) * 1e3, statistics.median(b[1:]) * 1e3


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else min(8, os.cpu_count() or 1)
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.set_num_threads(threads)
    host = {"cpu": cpu_model(), "threads": threads, "os_cpus": os.cpu_count(),
            "torch": torch.__version__}
    fwd, bwd = time_ntxent()
    print(json.dumps({"what": "ntxent B=512 C=256", "fwd_ms": round(fwd, 1), "bwd_ms": round(bwd, 1),
                      "survey_fwd_ms": [320, 390], "survey_bwd_ms": [2300, 2800], **host}),
          flush=True)
    for name, (kind, L, D, B, band) in CFG.items():
        ms = time_step(kind, L, D, B, steps if name != "c1" else 10)
        mid = 0.5 * (band[0] + band[1])
        print(json.dumps({"config": name, "ms_per_step": round(ms, 1), "survey_ms": list(band),
                          "ratio_to_survey_mid": round(ms / mid, 3),
                          "within_20pct": abs(ms / mid - 1) <= 0.2, **host}), flush=True)


if __name__ == "__main__":
    main()
