"""bf16 GEMM shapes of the c5 step (GIN 5x512, paired views, ~55k rows):
molclr_gemm_bf16_impl / molclr_linear_wgrad_bf16_impl tile shapes vs torch.matmul on bf16
(hipBLASLt).  Prints microseconds and TFLOP/s per shape.

    python tools/gemm_bf16_bench.py [rows]
"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
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
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 55342
    D, H = 512, 1024
    bf = torch.bfloat16
    torch.manual_seed(0)
    agg = torch.randn(M, D, device=dev).to(bf)
    a1 = torch.randn(M, H, device=dev).relu_().to(bf)
    dz = torch.randn(M, D, device=dev).to(bf)
    dz1 = torch.randn(M, H, device=dev).to(bf)
    W0 = torch.randn(H, D, device=dev) * 0.05
    W2 = torch.randn(D, H, device=dev) * 0.05
    b0, b2 = torch.randn(H, device=dev), torch.randn(D, device=dev)
    p0 = ops.weight_planes(W0, H, D, D, 0)      # x W0^T
    p2 = ops.weight_planes(W2, D, H, H, 0)      # a1 W2^T
    p2t = ops.weight_planes(W2, H, D, H, 1)     # dz W2
    p0t = ops.weight_planes(W0, D, H, D, 1)     # dz1 W0
    out_h = torch.empty(M, H, dtype=bf, device=dev)
    out_d = torch.empty(M, D, dtype=bf, device=dev)
    st = _lib.stream_of(dev)
    W0b, W2b = W0.to(bf), W2.to(bf)
    cases = [
        ("lin1 fwd agg W0^T+b relu", agg, p0, out_h, H, D, EPI_BIAS_RELU, b0, None,
         lambda: torch.addmm(b0.to(bf), agg, W0b.t()).relu_()),
        ("lin2 fwd a1 W2^T+b", a1, p2, out_d, D, H, EPI_BIAS, b2, None,
         lambda: torch.addmm(b2.to(bf), a1, W2b.t())),
        ("dz1 = dz W2 * (a1>0)", dz, p2t, out_h, H, D, EPI_RELU_MASK, None, a1,
         lambda: (dz @ W2b).mul_(a1 > 0)),
        ("dagg = dz1 W0", dz1, p0t, out_d, D, H, EPI_NONE, None, None, lambda: dz1 @ W0b),
        # the lin1 / dz1 shapes without their epilogues: what the epilogue costs
        ("lin1 shape, no epilogue", agg, p0, out_h, H, D, EPI_NONE, None, None,
         lambda: agg @ W0b.t()),
    ]
    for name, A, P, C, N, K, epi, bias, aux, ref in cases:
        fl = 2.0 * M * N * K
        res = []
        for v in (int(a) for a in os.environ.get("IMPLS", "6,8,9").split(",")):
            t = timeit(lambda: lib.molclr_gemm_bf16_impl(A.data_ptr(), P.data_ptr(), C.data_ptr(), M,
                                                         N, K, K, N, epi, _lib.ptr(bias),
                                                         _lib.ptr(aux), N if aux is not None else 0,
                                                         st, v))
            r = ref().float()
            err = ((C.float() - r).norm() / r.norm()).item()
            res.append(f"qb i{v} {t*1e6:6.1f}us {fl/t/1e12:6.1f}TF e{err:.0e}")
        t = timeit(ref)
        print(f"{name:26s} " + " | ".join(res) + f" | torch {t*1e6:6.1f}us {fl/t/1e12:6.1f}TF",
              flush=True)
    for name, dy, x, n_out, n_in in (("dW2 = dz^T a1 (+db)", dz, a1, D, H),
                                     ("dW0 = dz1^T agg (+db)", dz1, agg, H, D)):
        fl = 2.0 * M * n_out * n_in
        ws_bytes = lib.molclr_linear_wgrad_bf16_workspace_bytes(M, n_out, n_in)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        dW = torch.empty(n_out, n_in, device=dev)
        db = torch.empty(n_out, device=dev)
        res = []
        for v in (1, 3):
            t = timeit(lambda: lib.molclr_linear_wgrad_bf16_impl(
                dy.data_ptr(), x.data_ptr(), dW.data_ptr(), db.data_ptr(), M, n_out, n_in, n_out,
                n_in, 0, ws.data_ptr(), ws_bytes, st, v))
            r = dy.float().t() @ x.float()
            err = ((dW - r).norm() / r.norm()).item()
            rb = dy.float().sum(0)
            errb = ((db - rb).norm() / rb.norm()).item()
            res.append(f"wb i{v} {t*1e6:6.1f}us {fl/t/1e12:6.1f}TF e{err:.0e}/{errb:.0e}")
        t = timeit(lambda: dy.t() @ x)
        print(f"{name:26s} " + " | ".join(res) + f" | torch {t*1e6:6.1f}us {fl/t/1e12:6.1f}TF",
              flush=True)


if __name__ == "__main__":
    main()
