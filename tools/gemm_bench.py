"""GEMM shapes of the c2 step: molclr_gemm_f32 vs torch.matmul (hipBLASLt /
rocBLAS fp32) on the same operands.  Prints TFLOP/s per shape.

    python tools/gemm_bench.py [N_rows]
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
    cases = [
        ("lin1 fwd  x W1^T +b relu", 2 * Nr * H * D,
         lambda: ops.gemm(x, W1, Nr, H, D, D, D, 0, 0, EPI_BIAS_RELU, bias=b1),
         lambda: torch.addmm(b1, x, W1.t()).relu_()),
        ("lin2 fwd  a1 W2^T +b", 2 * Nr * H * D,
         lambda: ops.gemm(a1, W2, Nr, D, H, H, H, 0, 0, EPI_BIAS, bias=b2),
         lambda: torch.addmm(b2, a1, W2.t())),
        ("dz1 = dz W2 * (a1>0)", 2 * Nr * H * D,
         lambda: ops.gemm(dz, W2, Nr, H, D, D, H, 0, 1, EPI_RELU_MASK, aux=a1),
         lambda: (dz @ W2).mul_(a1 > 0)),
        ("dagg = dz1 W1", 2 * Nr * H * D,
         lambda: ops.gemm(dz1, W1, Nr, D, H, H, D, 0, 1),
         lambda: dz1 @ W1),
        ("dW2 = dz^T a1 (split-K)", 2 * Nr * H * D,
         lambda: ops.gemm(dz, a1, D, H, Nr, D, H, 1, 1),
         lambda: dz.t() @ a1),
        ("dW1 = dz1^T x (split-K)", 2 * Nr * H * D,
         lambda: ops.gemm(dz1, x, H, D, Nr, H, D, 1, 1),
         lambda: dz1.t() @ x),
    ]
    print(f"rows={Nr}  (fp32; torch.backends.cuda.matmul.allow_tf32="
          f"{torch.backends.cuda.matmul.allow_tf32})")
    from molclr_amd import _lib
    lib = _lib.load()
    for name, flops, mine, ref in cases:
        res = []
        for impl in (0, 1, 2, 3, 4):
            lib.molclr_gemm_set_impl(impl)
            tm = timeit(mine)
            res.append(f"impl{impl} {tm*1e6:6.1f}us {flops/tm/1e12:5.1f}TF")
        lib.molclr_gemm_set_impl(0)
        tr = timeit(ref)
        print(f"{name:26s} " + " | ".join(res) + f" | torch {tr*1e6:6.1f}us {flops/tr/1e12:5.1f}TF",
              flush=True)
    # correctness of every impl on one shape per layout
    torch.manual_seed(1)
    for impl in (1, 2, 3, 4):
        lib.molclr_gemm_set_impl(impl)
        for (ak, bk) in ((0, 0), (0, 1), (1, 1), (1, 0)):
            M, N, K = 333, 300, 1000
            Am = torch.randn(M, K, dtype=torch.float64)
            Bm = torch.randn(K, N, dtype=torch.float64)
            A = (Am.t() if ak else Am).contiguous().float().to(dev)
            Bt = (Bm if bk else Bm.t()).contiguous().float().to(dev)
            out = ops.gemm(A, Bt, M, N, K, M if ak else K, N if bk else K, ak, bk)
            ref = Am @ Bm
            err = ((out.double().cpu() - ref).norm() / ref.norm()).item()
            print(f"impl{impl} ak={ak} bk={bk} rel err {err:.2e}", flush=True)
            assert err < 1e-5
    lib.molclr_gemm_set_impl(0)


if __name__ == "__main__":
    main()
