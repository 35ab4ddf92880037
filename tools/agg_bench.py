"""Variants of the GINE forward aggregation on the c2 batches (tuning tool).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/aggvar.hip -o tools/libaggvar.so
    python tools/agg_bench.py

Prints mean per-launch kernel time (dispatch events) and the algorithmic
GB/s (ops.gine_aggregate_bytes) for each variant, after checking that each
is bit-identical to the library kernel.
"""
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import ops  # noqa: E402
from molclr_amd.data import device_graph  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402

NAMES = {0: "v0 library (CSR)", 1: "ELL int4, remap", 2: "ELL int4, no remap",
         3: "ELL int4, nt store", 4: "ELL int4, 2/thread", 5: "copy floor (no gather)",
         6: "ELL + combined table, nt", 7: "LDS tile R32 cap56", 8: "LDS tile R16 cap40",
         9: "LDS tile R64 cap96", 10: "LDS tile2 R32 cap48 512thr", 11: "LDS tile2 R16 cap32 512thr",
         12: "ELL + comb table, self last", 13: "ELL8 + comb table"}


def main():
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(str(ROOT / "tools" / "libaggvar.so"))
    lib.aggvar_run.restype = ctypes.c_double
    D = 300
    d4 = D // 4
    nb = 16
    gen = SyntheticPairBatches(512, seed=0)
    views = [v for a, b in gen.take(nb // 2) for v in (a, b)]
    torch.manual_seed(0)
    E1 = torch.randn(5, D, device=dev)
    E2 = torch.randn(3, D, device=dev)
    gs, xs, outs, ells, ells8 = [], [], [], [], []
    stream = torch.cuda.current_stream().cuda_stream
    for v in views:
        v = v.to(dev)
        g = device_graph(v)
        N = g.num_nodes
        gs.append(g)
        xs.append(torch.randn(N, D, device=dev))
        outs.append(torch.empty(N, D, device=dev))
        e = torch.empty(N * 4, dtype=torch.int32, device=dev)
        lib.aggvar_make_ell(ctypes.c_void_p(g.rowptr.data_ptr()), ctypes.c_void_p(g.col.data_ptr()),
                            ctypes.c_void_p(g.ecode.data_ptr()), ctypes.c_void_p(e.data_ptr()),
                            ctypes.c_int64(N), ctypes.c_void_p(stream))
        ells.append(e)
        e8 = torch.empty(N * 8, dtype=torch.int32, device=dev)
        lib.aggvar_make_ell8(ctypes.c_void_p(g.rowptr.data_ptr()), ctypes.c_void_p(g.col.data_ptr()),
                             ctypes.c_void_p(g.ecode.data_ptr()), ctypes.c_void_p(e8.data_ptr()),
                             ctypes.c_int64(N), ctypes.c_void_p(stream))
        ells8.append(e8)
    deg = torch.cat([g.rowptr[1:] - g.rowptr[:-1] for g in gs])
    print(f"views {nb}, mean N {sum(g.num_nodes for g in gs)/nb:.0f}, in-degree max {int(deg.max())}, "
          f"frac deg>4 {(deg > 4).float().mean().item():.2e}")

    P = lambda ts: (ctypes.c_void_p * nb)(*[t.data_ptr() for t in ts])  # noqa: E731
    Ns = (ctypes.c_int64 * nb)(*[g.num_nodes for g in gs])
    args = lambda v=0: (P(xs), P([g.rowptr for g in gs]), P([g.col for g in gs]),  # noqa: E731
                    P([g.ecode for g in gs]), P(ells8 if v == 13 else ells), Ns, ctypes.c_void_p(E1.data_ptr()),
                    ctypes.c_void_p(E2.data_ptr()), P(outs), ctypes.c_int(d4),
                    ctypes.c_void_p(stream))
    def tile_ptr(g, R):
        gp = g.graph_ptr.long()
        a = torch.arange(0, (g.num_nodes + R - 1) // R + 1, device=dev) * R
        idx = torch.searchsorted(gp, a.clamp(max=g.num_nodes))
        tp = gp[idx.clamp(max=gp.numel() - 1)]
        tp[0] = 0
        tp[-1] = g.num_nodes
        tp = torch.where(a >= g.num_nodes, torch.full_like(tp, g.num_nodes), tp)
        return tp.int().contiguous()
    tiles = {R: [tile_ptr(g, R) for g in gs] for R in (16, 32)}
    tile_arrs = {R: P(tiles[R]) for R in tiles}  # kept alive: the library stores the pointer
    gptr_arr = tile_arrs[32]
    Gs = (ctypes.c_int64 * nb)(*[g.num_graphs for g in gs])
    lib.aggvar_set_graphs(gptr_arr, Gs)
    lib.aggvar_run(0, 256, nb, 1, *args())
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]
    nbytes = sum(ops.gine_aggregate_bytes(g.num_nodes, D, g.num_edges) for g in gs) / nb
    src = torch.randn(max(g.num_nodes for g in gs), D, device=dev)
    for warm in (0, 1):
      print(["x cold (rotating)", "x rewritten before each launch, plain block order",
             "x rewritten before each launch, XCD-remapped block order"][warm])
      lib.aggvar_set_warm(ctypes.c_void_p(src.data_ptr() if warm else 0), ctypes.c_int(warm == 2))
      if warm:
          ref = [torch.empty_like(o) for o in outs]
          for i in range(nb):
              xs[i].copy_(src[:gs[i].num_nodes])
          lib.aggvar_run(0, 256, nb, 1, *args())
          torch.cuda.synchronize()
          ref = [o.clone() for o in outs]
      for v in (0, 6, 13, 5):
        lib.aggvar_set_graphs(tile_arrs[16 if v == 11 else 32], Gs)
        for block in ((256,) if v == 0 else (256,)):
          for o in outs:
              o.zero_()
          lib.aggvar_run(v, block, nb, 2, *args(v))  # warm + check
          torch.cuda.synchronize()
          same = all(torch.equal(a, b) for a, b in zip(outs, ref))
          us = lib.aggvar_run(v, block, nb, 20, *args(v))
          print(f"{NAMES[v]:28s} block {block:4d}: {us:7.2f} us  {nbytes / us / 1e3:7.1f} GB/s  "
                f"bit-exact={same}", flush=True)


def transpose_main():
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(str(ROOT / "tools" / "libaggvar.so"))
    lib.aggvar_transpose.restype = ctypes.c_double
    D, nb = 300, 16
    views = [v for a, b in SyntheticPairBatches(512, seed=0).take(nb // 2) for v in (a, b)]
    gs = [device_graph(v.to(dev)) for v in views]
    xs = [torch.randn(g.num_nodes, D, device=dev) for g in gs]
    outs = [torch.empty_like(x) for x in xs]
    src = torch.randn(max(g.num_nodes for g in gs), D, device=dev)
    P = lambda ts: (ctypes.c_void_p * nb)(*[t.data_ptr() for t in ts])  # noqa: E731
    Ns = (ctypes.c_int64 * nb)(*[g.num_nodes for g in gs])
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    arrs = [P(xs), P([g.rowptr_t for g in gs]), P([g.col_t for g in gs]), P([g.nbr_t for g in gs])]
    outp = P(outs)
    ref = None
    for warm in (0, 1):
        for v in (0, 1, 3, 4):
            us = lib.aggvar_transpose(v, nb, 20, *arrs, Ns, outp, D // 4,
                                      ctypes.c_void_p(src.data_ptr() if warm else 0), stream)
            torch.cuda.synchronize()
            if ref is None:
                ref = [o.clone() for o in outs]
            same = all(torch.equal(a, b) for a, b in zip(outs, ref))
            print(f"transpose {['csr', 'slot remap', 'slot', 'slot selflast', 'slot pairs'][v]:10s} warm={warm}: {us:6.2f} us same={same}",
                  flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "transpose":
        transpose_main()
        sys.exit(0)
    main()
