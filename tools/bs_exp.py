"""B-stationary h3 GEMM (tools/exp/bs_exp.hip) against the product kernel at
the c2 step's K = 300 products (lin1: agg [M,300] x W1^T -> a1 [M,600] with
bias + ReLU, its ReLU bits, max |a1|, row maxima and max |agg|; dz1: dz
[M,300] x W2 -> [M,600] with the ReLU mask from bits, row maxima, max):
per-launch time, and C / bits / maxima equal to the product's bit for bit.

    bash tools/exp/build_bs_exp.sh && python tools/bs_exp.py [groups...]
"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS_RELU, EPI_RELU_MASK  # noqa: E402


def timeit(fn, reps=20):
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


def main():
    # arguments: groups:variant pairs (variant: 0 = 8 waves, A 2 steps ahead; 1 = 3 ahead;
    # 2 = 12 waves; 3 = 16 waves)
    groups_list = [tuple(int(x) for x in v.split(':')) for v in sys.argv[1:]] or [(51, 0)]
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    exp = ctypes.CDLL(str(ROOT / "tools" / "exp" / "libbs_exp.so"))
    P, I, Ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    exp.bs_exp.argtypes = [Ci, Ci, P, P, P, I, I, I, I, I, I, I, P, P, I, P, P, P, P, P, Ci, P, P, I,
                           Ci, Ci, P]
    st = _lib.stream_of(dev)
    torch.manual_seed(0)
    M, D = 30556, 300
    H = 2 * D
    A = {"agg": torch.randn(M, D, device=dev) * torch.rand(M, 1, device=dev) * 4,
         "dz": torch.randn(M, D, device=dev) * torch.rand(M, 1, device=dev) * 1e-3}
    W1 = torch.randn(H, D, device=dev) * 0.05
    W2 = torch.randn(D, H, device=dev) * 0.05
    b1 = torch.randn(H, device=dev)
    bits_in = torch.randint(-2**31, 2**31 - 1, ((H + 31) // 32, M), dtype=torch.int32, device=dev)
    out = []
    # (name, A, W, b_kmajor, epilogue, bias, bits_in)
    for name, Ak, W, bk, epi, bias, bi in (("lin1", "agg", W1, 0, EPI_BIAS_RELU, b1, None),
                                          ("dz1", "dz", W2, 1, EPI_RELU_MASK, None, bits_in)):
        X = A[Ak]
        N, K = H, D
        rows = torch.empty(M, device=dev)
        slot = torch.zeros(ops.MAX_SLOT, device=dev)
        lib.molclr_absmax_rows_f32(X.data_ptr(), M, K, K, rows.data_ptr(), slot.data_ptr(), 1, st)
        planes = ops.weight_planes(W, N, K, K if not bk else N, bk, "h3")
        npad = (N + 127) // 128 * 128
        kp = (K + 31) // 32 * 32
        bmax = planes[2 * npad * kp:]
        C = torch.empty(M, N, device=dev)
        bits_o = torch.zeros((N + 31) // 32, M, dtype=torch.int32, device=dev)
        crow_p = torch.zeros(int(lib.molclr_gemm_row_parts(N)), M, device=dev)
        crow_b = torch.zeros((N + 127) // 128, M, device=dev)
        cmax = torch.zeros(ops.MAX_SLOT, device=dev)
        amo = torch.zeros(ops.MAX_SLOT, device=dev)

        def prod():
            rc = lib.molclr_gemm_f32_h3_bits(
                X.data_ptr(), rows.data_ptr(), 1, planes.data_ptr(), C.data_ptr(), M, N, K, K, N,
                epi, _lib.ptr(bias), None, 0, _lib.ptr(bi), cmax.data_ptr(), crow_p.data_ptr(),
                amo.data_ptr(), bits_o.data_ptr() if epi == EPI_BIAS_RELU else None, st)
            assert rc == 0, _lib.last_error()

        def bs(gv):
            groups, variant = gv
            rc = exp.bs_exp(epi, 2, X.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, kp,
                            npad, N, _lib.ptr(bias), None, 0, rows.data_ptr(), bmax.data_ptr(),
                            cmax.data_ptr(), crow_b.data_ptr(), amo.data_ptr(), 1,
                            bits_o.data_ptr() if epi == EPI_BIAS_RELU else None, _lib.ptr(bi), M,
                            groups, variant, st)
            assert rc == 0, rc

        def state():
            torch.cuda.synchronize()
            return (C.clone(), bits_o.clone(), cmax.max().item(), amo.max().item())

        for t in (cmax, amo, bits_o):
            t.zero_()
        prod()
        ref = state()
        ref_rows = crow_p.max(0).values.clone()
        fl = 2.0 * M * N * K
        tp = statistics.median(timeit(prod) for _ in range(5))
        rec = {"case": name, "M": M, "N": N, "K": K, "product_us": round(tp, 2),
               "product_h3_frac": round(fl * 3 / (tp * 1e-6) / 2.5e15, 4)}
        for g in groups_list:
            for t in (cmax, amo, bits_o, C):
                t.zero_()
            bs(g)
            got = state()
            same = (torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
                    and got[2] == ref[2] and got[3] == ref[3]
                    and torch.equal(crow_b.max(0).values, ref_rows))
            tb = statistics.median(timeit(lambda: bs(g)) for _ in range(5))
            rec[f"bs_{g[0]}_{g[1]}_us"] = round(tb, 2)
            rec[f"bs_{g[0]}_{g[1]}_bit_identical"] = bool(same)
            if not same:
                d = (got[0] - ref[0]).abs().max().item()
                rec[f"bs_{g[0]}_{g[1]}_maxdiff"] = d
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()
