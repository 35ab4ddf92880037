"""Cold-input GINE scatter-add figure.

The in-step roofline of molclr_gine_aggregate_fwd is cache-warm: its input h
was written by the BatchNorm launch right before it, so part of it can be
served from the 256 MB MALL.  This tool times the same launch at the c2 paired
shape over R rotated (input, output, graph) sets, > 600 MB in total, so every
launch reads an h, a neighbour-slot table and writes an output that no recent
launch touched:

    python tools/scatter_cold.py [sets] [reps] [warm|cold]
    python tools/scatter_cold.py [sets] [reps] exp [blocks_per_cu]
    python tools/scatter_cold.py [sets] [reps] rowmax

``exp`` times the layout variants of tools/exp/agg_exp.hip (build with
tools/exp/build_agg_exp.sh) on the same cold rotation, each checked
bit-for-bit against the product kernel's output.

Per launch it reports the average time (HIP events on the launch stream), the
algorithmic bytes (ops.gine_aggregate_bytes: 2*N*D*4 + 16*N) and the fraction
of 8 TB/s.  ``warm`` runs the same launch on set 0 only (the in-step-like
figure) for comparison.  Under rocprofv3 the kernel is k_gine_agg_fwd.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd.data import pair_graph  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402

PEAK_GBS = 8000.0
VARIANTS = (0, 1, 3, 6, 4, 50, 51, 52, 53)


def main():
    sets = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    mode = sys.argv[3] if len(sys.argv) > 3 else "cold"
    dev = torch.device("cuda", 0)
    _lib.load()
    D, B = 300, 512
    gen = SyntheticPairBatches(B, seed=7)
    graphs, hs, outs = [], [], []
    for s in range(sets):
        xi, xj = gen.take(1)[0]
        g = pair_graph(xi.to(dev), xj.to(dev))
        graphs.append(g)
        hs.append(torch.randn(g.num_nodes, D, device=dev))
        outs.append(torch.empty(g.num_nodes, D, device=dev))
    Ec = torch.randn(_lib.NUM_ECOMB, D, device=dev)
    st = ops._stream(Ec)
    total = sum(h.numel() * 4 * 2 + g.nbr.numel() * g.nbr.element_size() + g.rowptr.numel() * 4
                + g.col.numel() * 4 + g.ecode.numel() * g.ecode.element_size()
                for g, h in zip(graphs, hs))

    def launch(s):
        g = graphs[s]
        _lib.call("molclr_gine_aggregate_fwd", hs[s].data_ptr(), g.rowptr.data_ptr(),
                  g.col.data_ptr(), g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                  outs[s].data_ptr(), g.num_nodes, D, st)

    if mode == "exp":
        return experiments(graphs, hs, outs, Ec, st, D, reps,
                           int(sys.argv[4]) if len(sys.argv) > 4 else 8)
    if mode == "rowmax":
        return rowmax_cost(graphs, hs, outs, Ec, st, D, reps)
    order = list(range(sets)) if mode == "cold" else [0] * sets
    # flush: a 1 GB write between the set-up and the timed loop evicts the MALL
    flush = torch.empty(256 * 2**20, device=dev)
    for s in order:
        launch(s)
    flush.fill_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(dev)
    e0.record(stream)
    for _ in range(reps):
        for s in order:
            launch(s)
    e1.record(stream)
    torch.cuda.synchronize()
    n = reps * len(order)
    us = e0.elapsed_time(e1) * 1e3 / n
    alg = sum(ops.gine_aggregate_bytes(graphs[s].num_nodes, D, graphs[s].num_edges)
              for s in order) / len(order)
    gbs = alg / us / 1e3
    print(json.dumps({"kernel": "k_gine_agg_fwd", "mode": mode, "sets": sets,
                      "rotated_MB": round(total / 1e6, 1), "launches": n,
                      "avg_us": round(us, 2), "alg_bytes_per_launch": int(alg),
                      "achieved_GBs": round(gbs, 1), "frac_of_8TBs": round(gbs / PEAK_GBS, 3),
                      "avg_nodes": sum(graphs[s].num_nodes for s in order) // len(order)}),
          flush=True)


def rowmax_cost(graphs, hs, outs, Ec, st, D, reps):
    """The product entry points cold and warm: the plain aggregation, and
    molclr_gine_aggregate_fwd_rowmax (row maxima for the h3 forward) without
    and with the max slot."""
    sets = len(graphs)
    P = _lib.load().molclr_bn_row_parts(D)
    parts = [torch.empty(P, g.num_nodes, device=Ec.device) for g in graphs]
    slot = torch.zeros(ops.MAX_SLOT, device=Ec.device)
    flush = torch.empty(256 * 2**20, device=Ec.device)
    alg = sum(ops.gine_aggregate_bytes(g.num_nodes, D, g.num_edges) for g in graphs) / sets

    def plain(s):
        g = graphs[s]
        _lib.call("molclr_gine_aggregate_fwd", hs[s].data_ptr(), g.rowptr.data_ptr(),
                  g.col.data_ptr(), g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                  outs[s].data_ptr(), g.num_nodes, D, st)

    def rowmax(with_slot):
        def f(s):
            g = graphs[s]
            _lib.call("molclr_gine_aggregate_fwd_rowmax", hs[s].data_ptr(), g.rowptr.data_ptr(),
                      g.col.data_ptr(), g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                      outs[s].data_ptr(), g.num_nodes, D, parts[s].data_ptr(),
                      slot.data_ptr() if with_slot else None, st)
        return f
    for name, fn in (("plain", plain), ("rowmax", rowmax(False)), ("rowmax+slot", rowmax(True))):
        for mode in ("cold", "warm"):
            order = list(range(sets)) if mode == "cold" else [0] * sets
            for s in order:
                fn(s)
            flush.fill_(1.0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                for s in order:
                    fn(s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (reps * sets)
            print(json.dumps({"entry": name, "mode": mode, "avg_us": round(us, 2),
                              "frac_of_8TBs": round(alg / us / 1e3 / PEAK_GBS, 3)}), flush=True)


def experiments(graphs, hs, outs, Ec, st, D, reps, bpc):
    import ctypes
    lib = ctypes.CDLL(str(ROOT / "tools" / "exp" / "libagg_exp.so"))
    P, I = ctypes.c_void_p, ctypes.c_int64
    lib.agg_exp.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, I, I, ctypes.c_int, P]
    sets = len(graphs)
    ref = []
    for s in range(sets):
        g = graphs[s]
        _lib.call("molclr_gine_aggregate_fwd", hs[s].data_ptr(), g.rowptr.data_ptr(),
                  g.col.data_ptr(), g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                  outs[s].data_ptr(), g.num_nodes, D, st)
        ref.append(outs[s].clone())
    flush = torch.empty(256 * 2**20, device=Ec.device)
    alg = sum(ops.gine_aggregate_bytes(g.num_nodes, D, g.num_edges) for g in graphs) / sets
    names = {0: "product structure", 1: "copy floor (x -> out)", 2: "two units per thread",
             3: "non-temporal stores", 4: f"persistent {bpc}/CU + slot prefetch",
             5: "no XCD remap", 6: "empty kernel (launch floor)",
             7: "branch-free slots", 8: "branch-free, 2 units/thread",
             9: "branch-free + non-temporal",
             50: f"chunked persistent {bpc}/CU", 51: f"chunked copy floor {bpc}/CU",
             52: f"chunked persistent {bpc}/CU, non-temporal",
             53: f"chunked copy floor {bpc}/CU, non-temporal", 40: "branch-free, 2 units/thread, non-temporal",
             41: "branch-free, 4 units/thread, non-temporal"}
    for k, bs in ((10, 512), (20, 1024), (30, 128)):
        for b, w in list(names.items()):
            if b in (0, 1, 3, 6) and k + b in VARIANTS:
                names[k + b] = f"{w}, {bs}-thread blocks"
    for v in VARIANTS:
        def launch(s):
            g = graphs[s]
            rc = lib.agg_exp(v, hs[s].data_ptr(), g.rowptr.data_ptr(), g.col.data_ptr(),
                             g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                             outs[s].data_ptr(), g.num_nodes, D, bpc, st)
            assert rc == 0, rc
        for s in range(sets):
            outs[s].zero_()
            launch(s)
        torch.cuda.synchronize()
        copy = v in (1, 51, 53) or (v < 40 and v % 10 == 1)
        same = all(torch.equal(outs[s], ref[s] if not copy else hs[s])
                   for s in range(sets)) if v % 10 != 6 else None
        flush.fill_(1.0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            for s in range(sets):
                launch(s)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (reps * sets)
        print(json.dumps({"variant": v, "what": names[v], "avg_us": round(us, 2),
                          "frac_of_8TBs": round(alg / us / 1e3 / PEAK_GBS, 3),
                          "bit_exact": same}), flush=True)


if __name__ == "__main__":
    main()
