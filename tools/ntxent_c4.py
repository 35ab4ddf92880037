"""NT-Xent of one data-parallel rank at the c4 shape (BASELINE config 4):
rows [zj_local; zi_local] = 2 x 512, gathered columns 2 x 4096, C = 256 --
molclr_ntxent_prep, _fwd_impl (S kept) and _bwd_impl + _prep_bwd through the
C ABI, timed with HIP events (per step and per part), for rocprofv3 --stats.

    python tools/ntxent_c4.py [reps] [impl]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib  # noqa: E402
from molclr_amd import distributed as mdist  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    impl = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    st = _lib.stream_of(dev)
    W, Bl, C, T = 8, 512, 256, 0.1
    B, n = W * Bl, 2 * Bl
    torch.manual_seed(0)
    R = torch.randn(n, C, device=dev)
    cols = torch.nn.functional.normalize(torch.randn(2 * B, C, device=dev), dim=1)
    gidx = mdist.global_row_index(Bl, 0, W, dev)
    rh, nrm = torch.empty_like(R), torch.empty(n, device=dev)
    lse, lr = torch.empty(n, device=dev), torch.empty(n, device=dev)
    lse_cols = torch.randn(2 * B, device=dev).abs() + 5
    gl = torch.ones((), device=dev)
    drh, dR = torch.empty_like(R), torch.empty_like(R)
    wsb = lib.molclr_ntxent_workspace_bytes(n, 2 * B, C)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sb = lib.molclr_ntxent_sim_bytes(n, 2 * B, C, impl)
    sim = torch.empty(max(sb, 4), dtype=torch.uint8, device=dev) if sb else None

    def fwd():
        assert lib.molclr_ntxent_prep(R.data_ptr(), rh.data_ptr(), nrm.data_ptr(), n, C, 1, st) == 0
        assert lib.molclr_ntxent_fwd_impl(rh.data_ptr(), gidx.data_ptr(), cols.data_ptr(), n,
                                          2 * B, C, B, T, lse.data_ptr(), lr.data_ptr(),
                                          _lib.ptr(sim), ws.data_ptr(), wsb, st, impl) == 0

    def bwd():
        assert lib.molclr_ntxent_bwd_impl(rh.data_ptr(), gidx.data_ptr(), cols.data_ptr(),
                                          lse_cols.data_ptr(), gl.data_ptr(), n, 2 * B, C, B, T,
                                          _lib.ptr(sim), drh.data_ptr(), ws.data_ptr(), wsb, st,
                                          impl) == 0
        assert lib.molclr_ntxent_prep_bwd(drh.data_ptr(), rh.data_ptr(), nrm.data_ptr(),
                                          dR.data_ptr(), n, C, 1, st) == 0

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    tf, tb = timeit(fwd), timeit(bwd)
    flops = 2.0 * n * 2 * B * C
    print(f"c4 rank shard {n} x {2 * B} x {C} impl {impl}: fwd {tf:.1f} us, bwd {tb:.1f} us, "
          f"step {tf + tb:.1f} us; {3 * flops / (tf + tb) / 1e6:.1f} TF (S fwd + S-free bwd "
          f"as 2 products: {flops / 1e9:.2f} GFLOP each)", flush=True)


if __name__ == "__main__":
    main()
