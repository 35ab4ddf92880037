"""GEMM shapes of the c2 step: molclr_gemm_f32 vs torch.matmul (hipBLASLt /
rocBLAS fp32) on the same operands.  Prints TFLOP/s per shape.

    python tools/gemm_bench.py [N_rows] [impl,impl,...] [tile,tile,...]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import ops  # noqa: E402
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


def main():
    dev = torch.device("cuda", 0)
    Nr = int(sys.argv[1]) if len(sys.argv) > 1 else 15278
    D, H = 300, 600
    torch.manual_seed(0)
    x = torch.randn(Nr, D, device=dev)
    a1 = torch.randn(Nr, H, device=dev).relu_()
    dz = torch.randn(Nr, D, device=dev)
    dz1 = torch.randn(Nr, H, device=dev)
    W1 = torch.randn(H, D, device=dev)
    W2 = torch.randn(D, H, device=dev)
    b1 = torch.randn(H, device=dev)
    b2 = torch.randn(D, device=dev)
    # (name, A, B, M, N, K, lda, ldb, ak, bk, epi, kwargs, B is a weight, torch reference)
    cases = [
        ("lin1 fwd  x W1^T +b relu", x, W1, Nr, H, D, D, D, 0, 0, EPI_BIAS_RELU, dict(bias=b1), True,
         lambda: torch.addmm(b1, x, W1.t()).relu_()),
        ("lin2 fwd  a1 W2^T +b", a1, W2, Nr, D, H, H, H, 0, 0, EPI_BIAS, dict(bias=b2), True,
         lambda: torch.addmm(b2, a1, W2.t())),
        ("dz1 = dz W2 * (a1>0)", dz, W2, Nr, H, D, D, H, 0, 1, EPI_RELU_MASK, dict(aux=a1), True,
         lambda: (dz @ W2).mul_(a1 > 0)),
        ("dagg = dz1 W1", dz1, W1, Nr, D, H, H, D, 0, 1, 0, {}, True, lambda: dz1 @ W1),
        ("dW2 = dz^T a1 (split-K)", dz, a1, D, H, Nr, D, H, 1, 1, 0, {}, False, lambda: dz.t() @ a1),
        ("dW1 = dz1^T x (split-K)", dz1, x, H, D, Nr, H, D, 1, 1, 0, {}, False, lambda: dz1.t() @ x),
    ]
    print(f"rows={Nr}  (fp32; torch.backends.cuda.matmul.allow_tf32="
          f"{torch.backends.cuda.matmul.allow_tf32})")
    from molclr_amd import _lib
    lib = _lib.load()
    impls = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else "-1,0,5,6".split(","))]
    tiles = [int(v) for v in (sys.argv[3].split(",") if len(sys.argv) > 3 else "5,7,9".split(","))]
    for name, A, B, M, N, K, lda, ldb, ak, bk, epi, kw, weight, ref in cases:
        flops = 2 * M * N * K
        res = []
        for impl in impls:
            tm = timeit(lambda: ops.gemm(A, B, M, N, K, lda, ldb, ak, bk, epi, impl=impl, **kw))
            res.append(f"i{impl} {tm*1e6:5.1f}us {flops/tm/1e12:5.1f}TF")
        if ak and bk:  # weight gradient: the long-K kernel with one / two K groups
            ws_bytes = lib.molclr_linear_wgrad_workspace_bytes(K, M, N)
            ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
            out = torch.empty(M, N, device=dev)
            for kg in (1, 2):
                tm = timeit(lambda: lib.molclr_linear_wgrad_groups(
                    A.data_ptr(), B.data_ptr(), out.data_ptr(), None, K, M, N, lda, ldb, 0,
                    ws.data_ptr(), ws_bytes, _lib.stream_of(dev), kg))
                res.append(f"w6/kg{kg} {tm*1e6:5.1f}us {flops/tm/1e12:5.1f}TF")
        if weight:
            for t in tiles:
                tm = timeit(lambda: ops.gemm_w(A, B, M, N, K, lda, ldb, ak, bk, epi, tile=t, **kw))
                res.append(f"bp{t} {tm*1e6:5.1f}us {flops/tm/1e12:5.1f}TF")
        tr = timeit(ref)
        print(f"{name:24s} " + " | ".join(res) + f" | torch {tr*1e6:5.1f}us {flops/tr/1e12:5.1f}TF",
              flush=True)


if __name__ == "__main__":
    main()
