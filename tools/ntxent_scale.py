"""NT-Xent kernel cost per rank as the data-parallel world grows (c4 shape):
rank-local rows 2*512, gathered columns 2*512*W, C = 256.  Times
molclr_ntxent_fwd + _bwd on one GPU for W = 1, 2, 4, 8 (what one rank runs)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    Bl, C, T = 512, 256, 0.1
    st = _lib.stream_of(dev)
    for W in (1, 2, 4, 8):
        B = Bl * W
        n = 2 * Bl
        cols = torch.nn.functional.normalize(torch.randn(2 * B, C, device=dev), dim=1)
        rhat = torch.cat([cols[:Bl], cols[B:B + Bl]]).contiguous()
        base = torch.arange(Bl, dtype=torch.int32, device=dev)
        gidx = torch.cat([base, base + B])
        lse = torch.empty(n, device=dev)
        lr = torch.empty(n, device=dev)
        lse_cols = torch.randn(2 * B, device=dev).abs() + 5
        gl = torch.ones((), device=dev)
        dr = torch.empty_like(rhat)
        ws_bytes = _lib.query("molclr_ntxent_workspace_bytes", n, 2 * B, C)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)

        for impl in (0, 1):
            sb = _lib.query("molclr_ntxent_sim_bytes", n, 2 * B, C, impl)
            sim = torch.empty(max(sb, 4), dtype=torch.uint8, device=dev) if sb else None

            def fwd():
                _lib.call("molclr_ntxent_fwd_impl", rhat.data_ptr(), gidx.data_ptr(),
                          cols.data_ptr(), n, 2 * B, C, B, T, lse.data_ptr(), lr.data_ptr(),
                          _lib.ptr(sim), ws.data_ptr(), ws_bytes, st, impl)

            def bwd():  # with the forward's S kept (formulation 1)
                _lib.call("molclr_ntxent_bwd_impl", rhat.data_ptr(), gidx.data_ptr(),
                          cols.data_ptr(), lse_cols.data_ptr(), gl.data_ptr(), n, 2 * B, C, B, T,
                          _lib.ptr(sim), dr.data_ptr(), ws.data_ptr(), ws_bytes, st, impl)
            from tools_gemm import timeit  # noqa: F401
            tf = timeit(fwd)
            tb = timeit(bwd)
            flops = 2.0 * n * 2 * B * C
            print(f"W={W} impl {impl}: cols {2 * B:5d}  fwd {tf * 1e6:7.1f} us "
                  f"({flops / tf / 1e12:5.1f} TF)  bwd {tb * 1e6:7.1f} us "
                  f"({2 * flops / tb / 1e12:5.1f} TF)", flush=True)


if __name__ == "__main__":
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import gemm_bench
    sys.modules["tools_gemm"] = gemm_bench
    main()
