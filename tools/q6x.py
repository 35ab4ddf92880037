"""q6 main-loop variants (tools/exp/q6x.hip) at the c2 step's four shapes:
per-launch time of each variant, bit-for-bit equality with variant 0 (a copy
of the product kernel), and the product kernel itself for reference.

    bash tools/exp/build_q6x.sh && python tools/q6x.py [variants...]
"""
import ctypes
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS, EPI_BIAS_RELU, EPI_NONE, EPI_RELU_MASK  # noqa: E402


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
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    variants = [int(v) for v in sys.argv[1:]] or [0, 1, 2, 3, 4, 7]
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    exp = ctypes.CDLL(str(ROOT / "tools" / "exp" / "libq6x.so"))
    P, I, Ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    exp.q6x.argtypes = [Ci, Ci, Ci, P, P, P, I, I, I, I, I, I, I, P, P, I, P, P, P, P, P, Ci, P, P,
                        I, P]
    st = _lib.stream_of(dev)
    torch.manual_seed(0)
    M, D = 30556, 300
    H = 2 * D
    X = {n: torch.randn(M, c, device=dev) for n, c in (("agg", D), ("a1", H), ("dz", D), ("dz1", H))}
    W0 = torch.randn(H, D, device=dev) * 0.05
    W2 = torch.randn(D, H, device=dev) * 0.05
    b0, b2 = torch.randn(H, device=dev), torch.randn(D, device=dev)
    bits = torch.randint(-2**31, 2**31 - 1, ((H + 31) // 32, M), dtype=torch.int32, device=dev)
    rmax = {}
    for n in ("dz", "dz1"):
        r = torch.empty(M, device=dev)
        slot = torch.zeros(ops.MAX_SLOT, device=dev)
        lib.molclr_absmax_rows_f32(X[n].data_ptr(), M, X[n].shape[1], X[n].shape[1], r.data_ptr(),
                                   slot.data_ptr(), 1, st)
        rmax[n] = r
    cases = []
    # (name, A, W, N, K, b_kmajor, epi, bias, h3 form, row maxima, bits in)
    cases.append(("lin1 x6", X["agg"], W0, H, D, 0, EPI_BIAS_RELU, b0, 0, None, None))
    cases.append(("lin2 x6", X["a1"], W2, D, H, 0, EPI_BIAS, b2, 0, None, None))
    cases.append(("dz1 h3", X["dz"], W2, H, D, 1, EPI_RELU_MASK, None, 2, rmax["dz"], bits))
    cases.append(("dagg h3", X["dz1"], W0, D, H, 1, EPI_NONE, None, 2, rmax["dz1"], None))
    for name, A, W, N, K, bk, epi, bias, h3, rm, bi in cases:
        planes = ops.weight_planes(W, N, K, K if not bk else N, bk, "h3" if h3 else "x6")
        npad = (N + 127) // 128 * 128
        kp = (K + 31) // 32 * 32
        bmax = planes[2 * npad * kp:] if h3 else None
        C = torch.empty(M, N, device=dev)
        # the step's side outputs: lin1 writes a1's ReLU bits, max |a1| and
        # max |agg|; dz1 writes dz1's row maxima per column tile and max |dz1|
        bits_o = torch.zeros((N + 31) // 32, M, dtype=torch.int32, device=dev) if name.startswith("lin1") else None
        crow = torch.zeros((N + 159) // 160, M, device=dev) if name.startswith("dz1") else None
        cmax = torch.zeros(ops.MAX_SLOT, device=dev) if name.startswith(("lin1", "dz1")) else None
        amo = torch.zeros(ops.MAX_SLOT, device=dev) if name.startswith("lin1") else None

        def run(v):
            for t in (bits_o, crow, cmax, amo):
                if t is not None:
                    t.zero_()
            rc = exp.q6x(v, epi, h3, A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, kp,
                         npad, N, _lib.ptr(bias), None, 0, _lib.ptr(rm),
                         bmax.data_ptr() if bmax is not None else None, _lib.ptr(cmax),
                         _lib.ptr(crow), _lib.ptr(amo), 1 if h3 else 0, _lib.ptr(bits_o),
                         _lib.ptr(bi), M, st)
            assert rc == 0, (v, rc)

        def outs():
            # max slots: compare their maxima (entries depend on the block count)
            return [C.clone()] + [t.clone() for t in (bits_o, crow) if t is not None] + \
                [t.max().reshape(1) for t in (cmax, amo) if t is not None]

        if h3:
            prod = lambda: lib.molclr_gemm_f32_h3(  # noqa: E731
                A.data_ptr(), rm.data_ptr(), 1, planes.data_ptr(), C.data_ptr(), M, N, K, K, N,
                epi, _lib.ptr(bias), None, 0, _lib.ptr(bi), None, None, None, st)
        else:
            wsb = lib.molclr_gemm_f32_workspace_bytes(M, N, K)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            prod = lambda: lib.molclr_gemm_f32_bplanes_tile(  # noqa: E731
                A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, N, 0, epi,
                _lib.ptr(bias), None, 0, ws.data_ptr(), wsb, st, 9)
        run(0)
        torch.cuda.synchronize()
        ref = outs()
        prod()
        torch.cuda.synchronize()
        same_prod = torch.equal(C, ref[0])
        same = {}
        for v in variants:
            C.zero_()
            run(v)
            torch.cuda.synchronize()
            same[v] = all(torch.equal(a, b) for a, b in zip(outs(), ref))
        times = {v: [] for v in variants}
        tp = []
        for _ in range(5):
            tp.append(timeit(prod))
            for v in variants:
                times[v].append(timeit(lambda: run(v)))
        fl = 2.0 * M * N * K
        line = f"{name:8s} product {statistics.median(tp):6.1f} us (v0 == product: {same_prod})"
        for v in variants:
            t = statistics.median(times[v])
            line += f" | v{v} {t:6.1f} us {fl / t / 1e6:5.1f} TF {'=' if same[v] else 'DIFF'}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
