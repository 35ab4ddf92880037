"""Where the q6 / h3 GEMM time goes on the c2 shapes: per-launch time of
molclr_gemm_f32_bplanes_tile (q6, tile 9) and molclr_gemm_f32_h3 as the
epilogue, K and output width vary, so the per-tile overhead (prologue +
epilogue) separates from the per-K-step cost.

    python tools/q6_exp.py [rows]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS, EPI_BIAS_RELU, EPI_NONE, EPI_RELU_MASK  # noqa: E402


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


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 30556
    st = _lib.stream_of(dev)
    torch.manual_seed(0)
    rows = []
    for (N, K) in ((600, 300), (300, 600), (600, 600), (300, 300), (600, 150), (1200, 300)):
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        aux = torch.randn(M, N, device=dev)
        C = torch.empty(M, N, device=dev)
        planes = ops.weight_planes(W, N, K, K, 0)
        hpl = ops.weight_planes(W, N, K, K, 0, "h3")
        ws_b = lib.molclr_gemm_f32_workspace_bytes(M, N, K)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        slots = torch.zeros(3, 2048, device=dev)
        rmax = torch.zeros(8, M, device=dev)
        bits = torch.zeros((N + 31) // 32, M, dtype=torch.int32, device=dev)
        amax = ops.absmax(A)
        arow = A.abs().amax(1).contiguous()
        fl = 2.0 * M * N * K
        res = {}
        for nm, epi, bias, ax in (("none", EPI_NONE, None, None), ("bias", EPI_BIAS, b, None),
                                  ("brelu", EPI_BIAS_RELU, b, None),
                                  ("mask", EPI_RELU_MASK, None, aux)):
            t = timeit(lambda: lib.molclr_gemm_f32_bplanes_tile(
                A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, N, 0, epi,
                _lib.ptr(bias), _lib.ptr(ax), N if ax is not None else 0, ws.data_ptr(), ws_b, st, 9))
            res["x6 " + nm] = t
        # the encoder's forward product: bias + ReLU with max slots, row maxima and ReLU bits
        t = timeit(lambda: lib.molclr_gemm_f32_bplanes_max(
            A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, N, EPI_BIAS_RELU,
            b.data_ptr(), None, 0, slots[0].data_ptr(), slots[1].data_ptr(), None,
            bits.data_ptr(), ws.data_ptr(), ws_b, st))
        res["x6 brelu+max+bits"] = t
        for nm, epi, mb in (("none", EPI_NONE, None), ("mask-bits", EPI_RELU_MASK, bits)):
            t = timeit(lambda: lib.molclr_gemm_f32_h3(
                A.data_ptr(), arow.data_ptr(), 1, hpl.data_ptr(), C.data_ptr(), M, N, K, K, N,
                epi, None, aux.data_ptr() if epi == EPI_RELU_MASK else None,
                N if epi == EPI_RELU_MASK else 0, _lib.ptr(mb), slots[2].data_ptr(),
                rmax.data_ptr(), None, st))
            res["h3 rows " + nm] = t
        tt = timeit(lambda: torch.matmul(A, W.t()))
        res["torch fp32"] = tt
        line = f"M={M} N={N:4d} K={K:4d} " + " | ".join(
            f"{k} {v*1e6:6.1f}us {fl/v/1e12:5.1f}TF" for k, v in res.items())
        print(line, flush=True)
        rows.append(line)
        del A, W, aux, C


if __name__ == "__main__":
    main()
