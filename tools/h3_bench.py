"""The c2 GIN-MLP GEMM shapes, split-bf16 x6 (q6 / w6) against the fp16 h3
form (three MFMAs): time per launch and norm-wise error against fp64.

    python tools/h3_bench.py [N_rows]
"""
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib  # noqa: E402
from molclr_amd._lib import EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_MASK  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def rel(a, ref):
    return ((a.double() - ref).norm() / ref.norm().clamp_min(1e-300)).item()


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    st = _lib.stream_of(dev)
    Nr = int(sys.argv[1]) if len(sys.argv) > 1 else 30556
    D, H = 300, 600
    g = torch.Generator(device="cpu").manual_seed(0)
    mk = lambda *s, scale=1.0: (torch.randn(*s, generator=g) * scale).to(dev)  # noqa: E731
    x = mk(Nr, D, scale=3.0)
    a1 = mk(Nr, H).relu_()
    dz = mk(Nr, D, scale=1e-5)     # gradients are small: the scaling must carry them
    dz1 = mk(Nr, H, scale=3e-6).mul_(a1 > 0)
    W1 = ((torch.rand(H, D, generator=g) * 2 - 1) / D ** 0.5).to(dev)
    W2 = ((torch.rand(D, H, generator=g) * 2 - 1) / H ** 0.5).to(dev)
    b1, b2 = mk(H, scale=0.05), mk(D, scale=0.05)

    def planes(fn_bytes, fn_make, B, N, K, kmajor):
        nb = getattr(lib, fn_bytes)(N, K)
        buf = torch.empty(nb, dtype=torch.uint8, device=dev)
        arrP = (ctypes.c_void_p * 1)(B.data_ptr())
        i64 = lambda v: (ctypes.c_int64 * 1)(v)  # noqa: E731
        rc = getattr(lib, fn_make)(1, arrP, i64(N), i64(K), i64(B.shape[1]),
                                   (ctypes.c_int * 1)(kmajor), (ctypes.c_void_p * 1)(buf.data_ptr()), st)
        assert rc == 0, lib.molclr_last_error()
        return buf

    def slot(t):
        s = torch.empty(2048, device=dev)
        lib.molclr_absmax_f32(t.data_ptr(), t.shape[0], t.shape[1], t.shape[1], s.data_ptr(), 0, st)
        return s

    smax = {id(t): slot(t) for t in (x, a1, dz, dz1)}
    fwd_cases = [
        # name, A, W, kmajor(W as B), N, K, epi, bias, aux, ref
        ("lin1 fwd x W1^T+b relu", x, W1, 0, H, D, EPI_BIAS_RELU, b1, None,
         lambda: torch.addmm(b1.double(), x.double(), W1.double().t()).relu()),
        ("lin2 fwd a1 W2^T+b", a1, W2, 0, D, H, EPI_BIAS, b2, None,
         lambda: torch.addmm(b2.double(), a1.double(), W2.double().t())),
        ("dz1 = dz W2 * (a1>0)", dz, W2, 1, H, D, EPI_RELU_MASK, None, a1,
         lambda: (dz.double() @ W2.double()) * (a1 > 0)),
        ("dagg = dz1 W1", dz1, W1, 1, D, H, 0, None, None, lambda: dz1.double() @ W1.double()),
    ]
    ws_b = max(lib.molclr_gemm_f32_workspace_bytes(Nr, H, H),
               lib.molclr_linear_wgrad_workspace_bytes(Nr, H, H))
    ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
    print(f"rows={Nr}")
    for name, A, W, km, N, K, epi, bias, aux, ref in fwd_cases:
        C6 = torch.empty(Nr, N, device=dev)
        C3 = torch.empty(Nr, N, device=dev)
        p6 = planes("molclr_bplanes_bytes", "molclr_bplanes_make_batch", W, N, K, km)
        p3 = planes("molclr_hplanes_bytes", "molclr_hplanes_make_batch", W, N, K, km)
        bp = bias.data_ptr() if bias is not None else None
        ap = aux.data_ptr() if aux is not None else None
        ld_aux = N if aux is not None else 0
        cmax = torch.zeros(2048, device=dev)

        def run6():
            rc = lib.molclr_gemm_f32_bplanes(A.data_ptr(), p6.data_ptr(), C6.data_ptr(), Nr, N, K, K,
                                             N, 0, epi, bp, ap, ld_aux, ws.data_ptr(), ws_b, st)
            assert rc == 0, lib.molclr_last_error()

        def run3():
            rc = lib.molclr_gemm_f32_h3(A.data_ptr(), smax[id(A)].data_ptr(), 0, p3.data_ptr(),
                                        C3.data_ptr(), Nr, N, K, K, N, epi, bp, ap, ld_aux, None,
                                        cmax.data_ptr(), None, None, st)
            assert rc == 0, lib.molclr_last_error()
        rws = torch.empty(Nr, device=dev)
        tmp_slot = torch.zeros(2048, device=dev)
        lib.molclr_absmax_rows_f32(A.data_ptr(), Nr, K, K, rws.data_ptr(), tmp_slot.data_ptr(), 1, st)
        C3r = torch.empty(Nr, N, device=dev)
        crow = torch.empty(lib.molclr_gemm_row_parts(N), Nr, device=dev)

        def run3r():  # row-wise A scales, C's row maxima out (the backward's form)
            rc = lib.molclr_gemm_f32_h3(A.data_ptr(), rws.data_ptr(), 1, p3.data_ptr(),
                                        C3r.data_ptr(), Nr, N, K, K, N, epi, bp, ap, ld_aux, None,
                                        cmax.data_ptr(), crow.data_ptr(), None, st)
            assert rc == 0, lib.molclr_last_error()
        t6, t3, t3r = timeit(run6), timeit(run3), timeit(run3r)
        r = ref()
        f32 = (A @ (W.t() if km == 0 else W))
        fl = 2 * Nr * N * K
        print(f"{name:24s} x6 {t6*1e6:6.1f}us ({fl/t6/1e12:5.1f}TF) err {rel(C6, r):.2e} | "
              f"h3 {t3*1e6:6.1f}us ({fl/t3/1e12:5.1f}TF) err {rel(C3, r):.2e} | "
              f"h3 row-wise {t3r*1e6:6.1f}us err {rel(C3r, r):.2e} | "
              f"torch fp32 matmul err {rel(f32 + (bias if bias is not None else 0), (A.double() @ (W.double().t() if km == 0 else W.double())) + (bias.double() if bias is not None else 0)):.2e}"
              f" | cmax {cmax.max().item():.4e} vs {C3.abs().max().item():.4e}", flush=True)
    wg_cases = [
        ("dW2 = dz^T a1 (+db2)", dz, a1, D, H),
        ("dW1 = dz1^T x (+db1)", dz1, x, H, D),
    ]
    for name, dy, X, n_out, n_in in wg_cases:
        dW6, dW3 = torch.empty(n_out, n_in, device=dev), torch.empty(n_out, n_in, device=dev)
        db6, db3 = torch.empty(n_out, device=dev), torch.empty(n_out, device=dev)

        def run6():
            rc = lib.molclr_linear_wgrad(dy.data_ptr(), X.data_ptr(), dW6.data_ptr(), db6.data_ptr(),
                                         Nr, n_out, n_in, n_out, n_in, 0, ws.data_ptr(), ws_b, st)
            assert rc == 0, lib.molclr_last_error()

        def run3():
            rc = lib.molclr_linear_wgrad_h3(dy.data_ptr(), smax[id(dy)].data_ptr(), X.data_ptr(),
                                            smax[id(X)].data_ptr(), dW3.data_ptr(), db3.data_ptr(),
                                            Nr, n_out, n_in, n_out, n_in, 0, ws.data_ptr(), ws_b, st)
            assert rc == 0, lib.molclr_last_error()
        def run3g1():
            rc = lib.molclr_linear_wgrad_h3_groups(
                dy.data_ptr(), smax[id(dy)].data_ptr(), X.data_ptr(), smax[id(X)].data_ptr(),
                dW3.data_ptr(), db3.data_ptr(), Nr, n_out, n_in, n_out, n_in, 0, ws.data_ptr(),
                ws_b, st, 1)
            assert rc == 0, lib.molclr_last_error()
        t6, t3, t3g1 = timeit(run6), timeit(run3), timeit(run3g1)
        print(f"   h3 wgrad one K group per block: {t3g1*1e6:6.1f}us")
        r = dy.double().t() @ X.double()
        rb = dy.double().sum(0)
        fl = 2 * Nr * n_out * n_in
        print(f"{name:24s} x6 {t6*1e6:6.1f}us ({fl/t6/1e12:5.1f}TF) err {rel(dW6, r):.2e} | "
              f"h3 {t3*1e6:6.1f}us ({fl/t3/1e12:5.1f}TF) err {rel(dW3, r):.2e} db {rel(db3, rb):.1e}"
              f" | torch fp32 err {rel(dy.t() @ X, r):.2e}", flush=True)


if __name__ == "__main__":
    main()
