"""Contrastive pre-training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c5] [--no-cpu-baseline]
                    [--augment host|device|subgraph|mix]

A step is the reference's hot-loop iteration (molclr.py:108-128): two
encoder forwards of augmented views, F.normalize, NT-Xent, backward, Adam —
including the per-batch graph build (the reference's add_self_loops work).
Inputs: NB distinct pre-built synthetic batches per rank, resident in HBM
before the timed region (SURVEY.md §8d generator; rank r uses seed r*10^6),
rotated every step so repeated steps do not re-read one batch.

Workloads: c2 = GIN 5x300, feat 512, batch 512 per GPU, fp32 (default; the
config the metric is quoted on); c1 = GIN 3x128, batch 64 (the reference's
CPU-runnable case: its CPU baseline is cheap); c3 = GCN 5x300; c5 = GIN 5x512, bf16
storage and MFMA with fp32 accumulation, batch 1024 per GPU, PubChem-shaped
graphs.  Both views run through one paired encoder pass with per-view
BatchNorm statistics (the reference's two calls).  N > 1 runs under torchrun,
one rank per GPU over RCCL: the NT-Xent batch is global (512 N), weak scaling.

The JSON line adds:
  roofline      — the GIN scatter-add (molclr_gine_aggregate_fwd; GCN's
                  molclr_gcn_aggregate_fwd for c3), HBM-bound:
                  algorithmic bytes per launch / mean kernel duration in the
                  timed region, against 8.0 TB/s.  Durations are the
                  dispatch-recorded events of hipExtLaunchKernelGGL
                  (molclr_ktimer_*), i.e. the kernel's own execution window.
  roofline_mfma — all encoder/head GEMM kernels (GEMM + split-K reduce), timed
                  over extra steps after the timed region, against 157.3 TF/s
                  (fp32 dense MFMA peak; fp32 configs, which run split-bf16
                  "x6" kernels, also report the fraction of their own ceiling
                  2.5 PF / 6) or 2.5 PF/s (bf16, c5).
  roofline_ntxent — every NT-Xent kernel (forward: S = R R^T as a split-bf16
                  GEMM + the row logsumexp; backward: the weights W from the
                  kept S and dR = W R), work = the two products' flops, against
                  157.3 TF/s (fp32 MFMA) and 417 TF/s (the six-product split-bf16
                  ceiling, 2.5 PF / 6); rows x cols x dim of this rank's share.
  roofline_ntxent_c4 — the same NT-Xent calls on one data-parallel rank's
                  share at c4 (BASELINE config 4: 8 ranks x 512 molecules ->
                  1024 rows x 8192 gathered columns x 256), standalone HIP
                  events over 20 fwd+bwd pairs on synthetic unit rows; the
                  automatic formulation there is h3 (three fp16 MFMAs per
                  product): frac against its ceiling 2.5 PF / 3.
  cpu_baseline  — the oracle (CPU restatement of the reference step, incl.
                  the broadcast-cosine NT-Xent) on this host, rank 0, N=1 only,
                  a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

METRIC = "contrastive pre-train molecules/sec at batch 512, 1/2/4/8 MI355X; HBM GB/s on scatter_add"
HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFS = 157.3

CONFIGS = {
    "c1": dict(model_type="gin", num_layer=3, emb_dim=128, feat_dim=512, batch=64,
               shape="uniform", desc="c1: GIN 3x128 feat 512, batch 64, 10-50 atom graphs "
                                     "(the reference's CPU-runnable case)"),
    "c2": dict(model_type="gin", num_layer=5, emb_dim=300, feat_dim=512, batch=512,
               shape="uniform", desc="c2: GIN 5x300 feat 512, batch 512/GPU, 10-50 atom graphs"),
    "c3": dict(model_type="gcn", num_layer=5, emb_dim=300, feat_dim=512, batch=512,
               shape="uniform", desc="c3: GCN 5x300 feat 512, batch 512/GPU, 10-50 atom graphs"),
    "c5": dict(model_type="gin", num_layer=5, emb_dim=512, feat_dim=512, batch=1024,
               shape="pubchem", precision="bf16",
               desc="c5: GIN 5x512 feat 512, bf16 (fp32 accumulation), batch 1024/GPU, "
                    "PubChem-shaped graphs (atoms ~ N(27, 9) clipped to [6, 80])"),
}
BF16_MFMA_PEAK_TFS = 2500.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--batches", type=int, default=16, help="distinct resident batches per rank")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--mfma-steps", type=int, default=10,
                   help="extra steps after the timed region with every GEMM launch timed")
    p.add_argument("--two-pass", action="store_true",
                   help="run the two views as two encoder calls (the reference's molclr.py:57,60) "
                        "instead of one paired pass with per-view BatchNorm statistics")
    p.add_argument("--augment", default="host", choices=("host", "device", "subgraph", "mix"),
                   help="host: pre-built resident batch pairs (default); device: both views "
                        "built inside every step by molclr_mask_views from a resident "
                        "molecule store; subgraph / mix: the same with molclr_aug_views "
                        "(dataset_subgraph.py / dataset_mix.py views)")
    p.add_argument("--dp", action="store_true",
                   help="at N = 1, run the data-parallel code path anyway (an RCCL group of one: "
                        "group NT-Xent, bucketed gradient all-reduce)")
    p.add_argument("--no-hip-graph", action="store_true",
                   help="run every step eagerly (host-enqueued launches) instead of replaying "
                        "the HIP graph captured per batch-size bucket (molclr_amd.graph_step; "
                        "paired pass only; N > 1 captures the RCCL collectives too)")
    return p.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(cfg, batches_cpu, steps):
    """Oracle step (reference restatement) timed on this host's cores, with its
    calibration against the survey's timing of the reference modules
    (tools/cpu_calibrate.py): the reference's own
    NT-Xent (utils/nt_xent.py, restated op for op and pinned by the goldens)
    is timed alone on the same host, and the step / NT-Xent ratio is compared
    with the survey's (c2: 3.8-4.2 s / 2.6-3.2 s = 1.19-1.62; c3 0.91-1.38).  A host slower
    than the survey's container scales both; the ratio says whether the
    restatement costs what the reference does."""
    import torch

    from oracle.reference_cpu import RefGCN, RefGINet, RefNTXentLoss, ref_train_step
    hw = host_cores()
    threads = hw["threads_used"]
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    M = RefGINet if cfg["model_type"] == "gin" else RefGCN
    model = M(cfg["num_layer"], cfg["emb_dim"], cfg["feat_dim"])
    crit = RefNTXentLoss("cpu", cfg["batch"], 0.1, True)
    opt = torch.optim.Adam(model.parameters(), 5e-4, weight_decay=1e-5)
    times = []
    for i in range(steps + 1):  # first step is warm-up
        xi, xj = batches_cpu[i % len(batches_cpu)]
        t0 = time.perf_counter()
        ref_train_step(model, crit, opt, xi, xj)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times[1:])
    out = {"value": round(cfg["batch"] / med, 2), "unit": "molecules/s", "cores": threads,
           "host": hw,
           "kind": "port", "ms_per_step": round(med * 1e3, 1),
           "sample": f"{steps} steps (+1 warm-up) of {cfg['desc']}, oracle/reference_cpu.py, "
                     f"torch CPU fp32, {threads} threads (one per physical core available "
                     f"to this process), median step"}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                out["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    if cfg["batch"] == 512:
        nt = []
        for _ in range(2):
            zi = torch.nn.functional.normalize(torch.randn(512, 256), dim=1).requires_grad_(True)
            zj = torch.nn.functional.normalize(torch.randn(512, 256), dim=1).requires_grad_(True)
            t0 = time.perf_counter()
            crit(zi, zj).backward()
            nt.append(time.perf_counter() - t0)
        ntx = min(nt)
        band = {"c2": [1.19, 1.62], "c3": [0.91, 1.38]}.get(cfg["desc"][:2])
        ratio = med / ntx
        # the restatement stands in for the reference's CPU path only while it
        # costs what the reference's modules do, relative to the reference's
        # own NT-Xent on the same host (say so in the line)
        out["calibrated"] = bool(band and band[0] <= ratio <= band[1])
        out["calibration"] = {
            "ntxent_fwd_bwd_ms": round(ntx * 1e3, 1),
            "step_over_ntxent": round(med / ntx, 3),
            "survey_step_over_ntxent": {"c2": [1.19, 1.62], "c3": [0.91, 1.38]}.get(
                cfg["desc"][:2]),
            "survey_ms_per_step": {"c2": [3800, 4200], "c3": [2900, 3600]}.get(
                cfg["desc"][:2]),
            "note": "survey timings: the reference modules on the 8-core build container; "
                    "tools/cpu_calibrate.py there gave c2 4844 ms / NT-Xent 3688 ms = 1.31"}
    return out


def host_cores() -> dict:
    """Physical cores of this host (unique (package, core) pairs of
    /proc/cpuinfo), the logical CPUs this process may run on (affinity) and
    the cgroup CPU quota; the CPU baseline uses one thread per physical core
    within the affinity set, capped by the quota (all physical
    cores; on a shared GPU box the job's share is what it can actually use)."""
    import math
    logical = os.cpu_count() or 1
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = list(range(logical))
    core_of, phys, cur = {}, set(), {}
    try:
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if "processor" in cur:
                    key = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                    core_of[int(cur["processor"])] = key
                    phys.add(key)
                cur = {}
                continue
            k, v = (t.strip() for t in line.split(":", 1))
            cur[k] = v
        if "processor" in cur:
            key = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
            core_of[int(cur["processor"])] = key
            phys.add(key)
    except OSError:
        pass
    phys_allowed = len({core_of[c] for c in allowed if c in core_of}) or len(allowed)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    used = phys_allowed if quota is None else max(1, min(phys_allowed, math.floor(quota)))
    return {"physical_cores": len(phys) or logical, "logical_cpus": logical,
            "affinity_cpus": len(allowed), "physical_cores_in_affinity": phys_allowed,
            "cgroup_cpu_quota": quota, "threads_used": used}


def split_ceiling(tfs, model_type) -> dict:
    """fp32 GEMMs: fraction of their own MFMA ceiling.  Forward products run as
    split-bf16 x6 (six bf16 MFMAs: 2.5 PF / 6); with ops.FP32_GEMM == "h3" the
    GIN backward products (4 of every layer's 6 equal-size products) run as h3
    (three fp16 MFMAs: 2.5 PF / 3), so the ceiling is their flop-weighted
    harmonic mean; with ops.H3_FORWARD (the default) the GIN forward products
    run as h3 too and the ceiling is h3's."""
    from molclr_amd import ops
    x6, h3 = BF16_MFMA_PEAK_TFS / 6, BF16_MFMA_PEAK_TFS / 3
    if model_type == "gin" and ops.FP32_GEMM == "h3" and ops.H3_FORWARD:
        ceil, form = h3, "h3"
    elif model_type == "gin" and ops.FP32_GEMM == "h3":
        ceil = 1.0 / ((2 / 6) / x6 + (4 / 6) / h3)
        form = "x6 forward, h3 backward"
    elif model_type == "gcn" and ops.FP32_GEMM == "h3":
        # GCN: one forward product per layer (x6), its weight and data
        # gradients in h3: 1 of every 3 equal-size products is x6
        ceil = 1.0 / ((1 / 3) / x6 + (2 / 3) / h3)
        form = "x6 forward, h3 backward"
    else:
        ceil, form = x6, "x6"
    return {"split_ceiling_tfs": round(ceil, 1), "split_form": form,
            "frac_of_split_ceiling": round(tfs / ceil, 4)}


def main():
    args = parse()
    import torch

    from molclr_amd import distributed as mdist
    from molclr_amd import ops
    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.optim import FusedAdam

    if args.dp and int(os.environ.get("WORLD_SIZE", 1)) == 1:
        # the data-parallel code path on one GPU: an RCCL process group of one
        import socket
        import torch.distributed as dist
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(s.getsockname()[1]))
        s.close()
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    rank, world, dev = mdist.init()
    if world != args.gpus:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
    cfg = CONFIGS[args.config]
    B = cfg["batch"]

    # ---- inputs: NB distinct batches, resident on the device -----------------
    t0 = time.perf_counter()
    gen = SyntheticPairBatches(B, seed=rank * 10**6, shape=cfg["shape"])
    batches_cpu = gen.take(args.batches)
    batches = [(a.to(dev), b.to(dev)) for a, b in batches_cpu]
    n_nodes = sum(a.x.shape[0] + b.x.shape[0] for a, b in batches_cpu) / (2 * len(batches_cpu))
    n_edges = sum(a.edge_index.shape[1] + b.edge_index.shape[1]
                  for a, b in batches_cpu) / (2 * len(batches_cpu))
    log(rank, f"built {args.batches} batches in {time.perf_counter() - t0:.1f}s "
              f"(mean N={n_nodes:.0f}, E={n_edges:.0f} per view)")

    # ---- model / optimiser / loss ---------------------------------------------
    torch.manual_seed(0)
    precision = cfg.get("precision", "fp32")
    if cfg["model_type"] == "gin":
        from molclr_amd.ginet_molclr import GINet
        model = GINet(cfg["num_layer"], cfg["emb_dim"], cfg["feat_dim"],
                      precision=precision).to(dev)
    else:
        from molclr_amd.gcn_molclr import GCN
        model = GCN(cfg["num_layer"], cfg["emb_dim"], cfg["feat_dim"]).to(dev)
    # parameters in gradient-bucket order: the overlapped all-reduce's buckets
    # are slices of the flat gradient buffer (DP only)
    # data-parallel code path: N > 1, or --dp at N = 1 (an RCCL group of one)
    dp = world > 1 or args.dp
    opt = FusedAdam(mdist.bucketed_parameters(model) if dp else model.parameters(), 5e-4,
                    weight_decay=1e-5)
    mdist.broadcast_params(opt.flat)
    reducer = (mdist.OverlappedGradReducer(model, opt, torch.distributed.group.WORLD)
               if dp and not args.two_pass else None)
    group = torch.distributed.group.WORLD if dp else None
    crit = NTXentLoss(dev, B * world, 0.1, True, group=group)

    store = None
    if args.augment != "host":
        # the un-augmented molecules of NB batches resident in HBM; every step
        # draws B of them and builds both views on the device
        from molclr_amd.augment import DeviceMoleculeStore
        import numpy as np
        nmol = args.batches * B
        store = DeviceMoleculeStore.from_molecules(
            SyntheticPairBatches(B, seed=rank * 10**6, shape=cfg["shape"]).molecules(nmol), dev)
        perm_rng = np.random.default_rng(rank * 10**6 + 3)
        id_sets = [perm_rng.permutation(nmol)[:B].astype(np.int64) for _ in range(args.batches)]
        id_sets_dev = [torch.from_numpy(v).to(dev) for v in id_sets]

    # the scatter-add timed for the HBM roofline: GINE's, or GCN's for c3
    agg_kind = "gcn_aggregate_fwd" if cfg["model_type"] == "gcn" else "gine_aggregate_fwd"
    captured = None
    if not args.two_pass and not args.no_hip_graph and mdist.graph_capturable():
        # N > 1: the step's RCCL collectives (NT-Xent all-gathers, bucketed
        # gradient all-reduces) are captured with it (a gloo group -- the
        # two-ranks-on-one-GPU test -- stays eager)
        from molclr_amd.graph_step import CapturedTrainStep
        captured = CapturedTrainStep(model, opt, crit, reducer=reducer)

    def step(i, eager=False):
        xi, xj = views_of(i)
        if captured is not None and not eager:
            # staging copy + one graph launch: the graph build, both views'
            # encoder pass, NT-Xent, backward and Adam replay on the device
            return captured(xi, xj)
        for g in (xi, xj):  # rebuild the graph every step: it is part of the work
            g.__dict__.pop("_molclr_graph", None)
            g.__dict__.pop("_molclr_pair_graph", None)
        opt.zero_grad()
        if reducer is not None:
            reducer.arm()
        if args.two_pass:
            _, zi = model(xi)
            _, zj = model(xj)
            loss = crit(ops.l2_normalize(zi), ops.l2_normalize(zj))
        else:  # both views in one pass (MolCLR._step's default)
            _, z = model.forward_pair(xi, xj)
            loss = crit.forward_pair_normalized(z)
        loss.backward()
        if reducer is not None:  # bucketed, overlapped with the encoder backward
            reducer.finish()
        elif dp:
            mdist.allreduce_grads(opt.flat_grad)
        opt.step()
        return loss

    def views_of(i):
        if store is None:
            return batches[i % len(batches)]
        k = i % len(id_sets)
        if args.augment == "device":
            return store.mask_views(id_sets_dev[k], seed=i, host_ids=id_sets[k])
        return store.aug_views(id_sets_dev[k], seed=i, mode=args.augment, host_ids=id_sets[k])

    if captured is not None:
        # capture every graph the run's batches need BEFORE the warm-up, so no
        # capture lands in the timed region: the resident batches, or (device
        # augmentation) the views of every step index the run will use
        t0 = time.perf_counter()
        if store is None:
            captured.prepare(batches)
        else:
            for i in list(range(args.warmup + args.steps + 3)):
                captured.prepare([views_of(i)])
        torch.cuda.synchronize()
        log(rank, f"captured {captured.captures} graphs in {time.perf_counter() - t0:.1f}s "
                  f"(node/edge capacities {sorted(captured.buckets)})")
    for i in range(args.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    log(rank, f"warm-up done, loss {loss.item():.4f}")
    # host cost of one step: enqueue time starting from an idle device (extra,
    # untimed steps; if it approaches ms_per_step the step is launch-bound)
    host = []
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step(args.warmup + args.steps + i)
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()

    # the timed region carries dispatch events on the scatter-add launches only
    # (10 per step); timing every GEMM launch too costs ~13 % of the step.  A
    # replayed graph cannot carry them: the scatter-add is then timed over
    # extra eager steps after the timed region, like the GEMMs
    timer = None if args.no_kernel_timing or captured is not None else \
        ops.KernelTimer(kinds=(agg_kind,))
    ops.set_kernel_timer(timer)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    captures_before = captured.captures if captured is not None else 0
    eager_before = captured.eager_steps if captured is not None else 0
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        loss = step(args.warmup + i)
        marks[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    captures_timed = (captured.captures - captures_before) if captured is not None else 0
    eager_timed = (captured.eager_steps - eager_before) if captured is not None else 0
    ops.set_kernel_timer(None)
    # every rank's view of the run (the first multi-GPU line must be readable
    # on its own): world size, graphs captured, captures and eager fallbacks
    # inside the timed region
    mine = torch.tensor([rank, world, captured.captures if captured is not None else 0,
                         captures_timed, eager_timed], dtype=torch.long, device=dev)
    if world > 1:
        allr = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(allr, mine)
    else:
        allr = [mine]
    per_rank = [dict(zip(("rank", "world_size", "captures", "captures_in_timed_region",
                          "eager_steps_in_timed_region"), (int(v) for v in t.tolist())))
                for t in allr]
    elapsed = mdist.max_over_ranks(elapsed, dev)
    final_loss = float(loss.item())

    ms_per_step = elapsed / args.steps * 1e3
    value = B * world * args.steps / elapsed
    # per-step device time between consecutive end-of-step events (no extra sync)
    step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
    median_ms = statistics.median(step_ms)

    # (the library keeps one timer: read the scatter-add samples before the GEMM pass)
    s = timer.summary() if timer is not None else {}
    agg_timing = "hipExtLaunchKernelGGL dispatch events in the timed region"
    if captured is not None and not args.no_kernel_timing and args.mfma_steps > 0:
        timer = ops.KernelTimer(kinds=(agg_kind,))
        ops.set_kernel_timer(timer)
        for i in range(args.mfma_steps):
            step(args.warmup + args.steps + 3 + i, eager=True)
        torch.cuda.synchronize()
        ops.set_kernel_timer(None)
        s = timer.summary()
        agg_timing = (f"hipExtLaunchKernelGGL dispatch events over {args.mfma_steps} eager steps "
                      f"after the timed region (the timed region replays HIP graphs)")
    # GEMM durations: dispatch events over extra steps after the timed region
    if timer is not None and args.mfma_steps > 0:
        gemm_timer = ops.KernelTimer(kinds=("gemm_f32", "ntxent"))
        ops.set_kernel_timer(gemm_timer)
        for i in range(args.mfma_steps):
            step(args.warmup + args.steps + 3 + i, eager=True)
        torch.cuda.synchronize()
        ops.set_kernel_timer(None)
        s.update({k: v for k, v in gemm_timer.summary().items() if k in ("gemm_f32", "ntxent")})

    roofline = roofline_mfma = roofline_ntxent = None
    if timer is not None:
        agg = s.get(agg_kind)
        if agg:
            per_launch_s = agg["ms"] / agg["launches"] / 1e3
            per_launch_bytes = agg["work"] / agg["launches"]
            achieved = per_launch_bytes / per_launch_s / 1e9
            roofline = {"kernel": ("molclr_gcn_aggregate_fwd (k_gcn_agg_fwd)" if agg_kind ==
                                   "gcn_aggregate_fwd" else
                                   ("molclr_gine_aggregate_fwd_bf16" if precision == "bf16" else
                                    "molclr_gine_aggregate_fwd_rowmax (+ its row maxima for the h3 "
                                    "forward)" if ops.H3_FORWARD else
                                    "molclr_gine_aggregate_fwd") + " (k_gine_agg_fwd)"),
                        "bound": "hbm",
                        "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": load_pmc_traffic(args.config, args.two_pass),
                        "bytes_per_launch": int(per_launch_bytes),
                        "us_per_launch": round(per_launch_s * 1e6, 2),
                        "launches": agg["launches"],
                        "timing": agg_timing}
        gm = s.get("gemm_f32")
        if gm:
            tfs = gm["work"] / (gm["ms"] / 1e3) / 1e12
            if precision == "bf16":
                peak, extra = BF16_MFMA_PEAK_TFS, {}
            else:
                # fp32 at fp32 accuracy from split bf16 / fp16 MFMAs: the
                # headline fraction is against that form's own ceiling; the
                # native fp32 MFMA peak is reported beside it
                sc = split_ceiling(tfs, cfg["model_type"])
                peak = sc["split_ceiling_tfs"]
                extra = {**sc, "fp32_mfma_peak": FP32_MFMA_PEAK_TFS,
                         "frac_of_fp32_mfma_peak": round(tfs / FP32_MFMA_PEAK_TFS, 4)}
            roofline_mfma = {"kernel": ("molclr_gemm_bf16 / _linear_wgrad_bf16 encoder GEMMs + "
                                        "the fp32 head GEMMs" if precision == "bf16" else
                                        "molclr_gemm_f32 (all launches)"), "bound": "mfma",
                             "achieved": round(tfs, 2), "peak": peak,
                             "unit": "TFLOP/s" + ("" if precision == "bf16" else
                                                  " (fp32-equivalent)"),
                             "frac": round(tfs / peak, 4),
                             "traffic": None, "launches": gm["launches"],
                             "ms_per_step": round(gm["ms"] / args.mfma_steps, 3),
                             **extra,
                             "timing": f"dispatch events over {args.mfma_steps} extra steps "
                                       f"after the timed region"}
        nx = s.get("ntxent")
        if nx:
            tfs = nx["work"] / (nx["ms"] / 1e3) / 1e12
            roofline_ntxent = {"kernel": "molclr_ntxent_fwd/_bwd: every kernel of both calls (the "
                                         "similarity GEMM S = R R^T, row logsumexp, weights W, "
                                         "dR = W R; split-bf16 MFMA)",
                               "bound": "mfma", "achieved": round(tfs, 2),
                               "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s (fp32-equivalent)",
                               "frac": round(tfs / FP32_MFMA_PEAK_TFS, 4),
                               "frac_of_split_bf16_ceiling": round(tfs / (BF16_MFMA_PEAK_TFS / 6), 4),
                               "traffic": None,
                               "rows": 2 * B,
                               "cols": 2 * B * world, "dim": cfg["feat_dim"] // 2,
                               "ms_per_step": round(nx["ms"] / args.mfma_steps, 3),
                               "timing": f"dispatch events over {args.mfma_steps} extra steps "
                                         f"after the timed region"}

    # the timed path against the eager step from the same state, on one of
    # the run's batches (outside the timed region): the replay
    # over its capacity bucket (padding rows) vs the batch at its own size
    parity = None
    if captured is not None:
        parity = captured.replay_vs_eager(*views_of(args.warmup))  # a prepared batch
        parity = {kk: (round(v, 9) if isinstance(v, float) else
                       [v[0], round(v[1], 9)] if isinstance(v, list) else v)
                  for kk, v in parity.items()}
        parity["check"] = ("CapturedTrainStep.replay_vs_eager: one step from the same state, "
                           "eager (own size) vs replayed (capacity bucket); "
                           "tests/test_gpu_bench_parity.py holds loss <= 1e-6, gradients "
                           "<= 1e-5 (bf16 1e-4) at this config")
        parity["ok"] = bool(parity["loss_rel"] <= 1e-6 and parity["grad_rel"] <= (
            1e-4 if precision == "bf16" else 1e-5) and parity["running_stats_rel"] <= 1e-6)

    roofline_ntxent_c4 = None
    if rank == 0 and not args.no_kernel_timing and precision != "bf16":
        roofline_ntxent_c4 = ntxent_c4_roofline(dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log(rank, "timing the CPU baseline (oracle) ...")
        # c5's oracle step (fp32, 2B = 2048 broadcast cosine) takes tens of
        # seconds: one timed step after the warm-up bounds the sample
        cpu = cpu_baseline(cfg, batches_cpu, 1 if args.config == "c5" else args.cpu_steps)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "molecules/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "median_ms_per_step": round(median_ms, 3),
            "median_value": round(B * world / (median_ms / 1e3), 1),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if precision == "bf16" else "f32",
            "data": f"synthetic: {args.batches} resident pre-built batch pairs per rank "
                    f"(SURVEY §8d generator, node-mask views), random-init weights",
            "config": {"workload": cfg["desc"], "model": f"{cfg['model_type']} "
                       f"{cfg['num_layer']}x{cfg['emb_dim']} feat {cfg['feat_dim']}",
                       "global_batch": B * world, "per_gpu_batch": B,
                       "mean_nodes_per_view": round(n_nodes), "mean_edges_per_view": round(n_edges),
                       "parallelism": f"dp{world}" + (" (RCCL group of one)" if dp and world == 1
                                                      else ""),
                       "views": ("two encoder calls (molclr.py:57,60)" if args.two_pass else
                                 "one paired encoder pass, per-view BatchNorm statistics"),
                       "launch": ("HIP graph per batch-size capacity bucket "
                                  "(molclr_amd.graph_step): captured before the warm-up, "
                                  "staged + replayed every step"
                                  if captured is not None else "eager (host-enqueued)"),
                       "augment": ("host: pre-built resident batch pairs" if store is None else
                                   "device: molclr_mask_views inside the step"
                                   if args.augment == "device" else
                                   f"device: molclr_aug_views ({args.augment}) inside the step")},
            "final_loss": round(final_loss, 5),
            "host_enqueue_ms_per_step": round(statistics.median(host) * 1e3, 3),
            "captures": captured.captures if captured is not None else 0,
            "captures_in_timed_region": captures_timed,
            "ranks": per_rank,
            "parity": parity,
            "roofline": roofline, "roofline_mfma": roofline_mfma,
            "roofline_ntxent": roofline_ntxent, "roofline_ntxent_c4": roofline_ntxent_c4,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if captured is not None:
        captured.close()  # graphs holding RCCL collectives go before their group
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


def ntxent_c4_roofline(dev, reps: int = 20) -> dict:
    """NT-Xent of one c4 data-parallel rank (rows [zj; zi] of 512 molecules,
    columns gathered from 8 ranks: 1024 x 8192 x 256) through the C ABI as the
    training step calls it: molclr_ntxent_prep, _fwd_impl (S kept), _bwd_impl,
    _prep_bwd.  Work = the two products S = R C^T and dR = W C."""
    import torch
    from molclr_amd import _lib
    from molclr_amd import distributed as mdist
    lib = _lib.load()
    st = _lib.stream_of(dev)
    W, Bl, C, T = 8, 512, 256, 0.1
    B, n = W * Bl, 2 * Bl
    g = torch.Generator(device=dev).manual_seed(4)
    R = torch.randn(n, C, device=dev, generator=g)
    cols = torch.nn.functional.normalize(torch.randn(2 * B, C, device=dev, generator=g), dim=1)
    gidx = mdist.global_row_index(Bl, 0, W, dev)
    rh, nrm = torch.empty_like(R), torch.empty(n, device=dev)
    lse, lr = torch.empty(n, device=dev), torch.empty(n, device=dev)
    lse_cols = torch.rand(2 * B, device=dev, generator=g) + 5
    gl = torch.ones((), device=dev)
    drh, dR = torch.empty_like(R), torch.empty_like(R)
    wsb = lib.molclr_ntxent_workspace_bytes(n, 2 * B, C)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sb = lib.molclr_ntxent_sim_bytes(n, 2 * B, C, -1)
    sim = torch.empty(max(sb, 4), dtype=torch.uint8, device=dev) if sb else None

    def pair():
        for rc in (lib.molclr_ntxent_prep(R.data_ptr(), rh.data_ptr(), nrm.data_ptr(), n, C, 1, st),
                   lib.molclr_ntxent_fwd_impl(rh.data_ptr(), gidx.data_ptr(), cols.data_ptr(), n,
                                              2 * B, C, B, T, lse.data_ptr(), lr.data_ptr(),
                                              _lib.ptr(sim), ws.data_ptr(), wsb, st, -1),
                   lib.molclr_ntxent_bwd_impl(rh.data_ptr(), gidx.data_ptr(), cols.data_ptr(),
                                              lse_cols.data_ptr(), gl.data_ptr(), n, 2 * B, C, B,
                                              T, _lib.ptr(sim), drh.data_ptr(), ws.data_ptr(), wsb,
                                              st, -1),
                   lib.molclr_ntxent_prep_bwd(drh.data_ptr(), rh.data_ptr(), nrm.data_ptr(),
                                              dR.data_ptr(), n, C, 1, st)):
            if rc != 0:
                raise RuntimeError(_lib.last_error())

    for _ in range(3):
        pair()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pair()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    work = (2 if sb else 3) * 2.0 * n * 2 * B * C  # S (again in the backward when not kept), dR
    tfs = work / (us / 1e6) / 1e12
    ceiling = BF16_MFMA_PEAK_TFS / 3
    return {"kernel": "molclr_ntxent_prep + _fwd_impl + _bwd_impl + _prep_bwd (automatic "
                      "formulation: h3 at this shape)", "bound": "mfma",
            "achieved": round(tfs, 2), "peak": round(ceiling, 1),
            "unit": "TFLOP/s (fp32-equivalent)", "frac": round(tfs / ceiling, 4),
            "frac_of_fp32_mfma_peak": round(tfs / FP32_MFMA_PEAK_TFS, 4), "traffic": None,
            "rows": n, "cols": 2 * B, "dim": C, "us_per_step": round(us, 1),
            "timing": f"HIP events around {reps} fwd+bwd pairs, standalone, after the timed region"}


def load_pmc_traffic(config: str, two_pass: bool):
    """HBM bytes per aggregation launch from the committed PMC summary of the
    same workload (profiles/*pmc_gine_agg_<config>[_pair].json, written by
    tools/pmc_traffic.py), or None."""
    tag = f"{config}{'' if two_pass else '_pair'}"
    cands = sorted((ROOT / "profiles").glob(f"*pmc_gine_agg_{tag}.json"))
    if not cands:
        return None
    try:
        return json.loads(cands[-1].read_text()).get("hbm_bytes_per_launch")
    except Exception:
        return None


if __name__ == "__main__":
    main()
