"""Run one GEMM shape of the c2 step with one molclr_gemm_f32 implementation
(for rocprofv3 PMC passes).   python tools/gemm_one.py [impl] [case] [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS_RELU  # noqa: E402


def main():
    impl = sys.argv[1] if len(sys.argv) > 1 else "1"
    bp = impl.startswith("bp")
    impl = int(impl[2:] if bp else impl)
    case = sys.argv[2] if len(sys.argv) > 2 else "lin1"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda", 0)
    Nr, D, H = 15278, 300, 600
    torch.manual_seed(0)
    x = torch.randn(Nr, D, device=dev)
    W1 = torch.randn(H, D, device=dev)
    b1 = torch.randn(H, device=dev)
    dz1 = torch.randn(Nr, H, device=dev)
    if bp:
        _lib.load().molclr_gemm_bplanes_set_impl(impl)
    else:
        _lib.load().molclr_gemm_set_impl(impl)
    for _ in range(reps):
        if case == "lin1":
            (ops.gemm_w if bp else ops.gemm)(x, W1, Nr, H, D, D, D, 0, 0, EPI_BIAS_RELU, bias=b1)
        else:  # dW1 = dz1^T x
            ops.gemm(dz1, x, H, D, Nr, H, D, 1, 1)
    torch.cuda.synchronize()
    print("done", impl, case, reps)


if __name__ == "__main__":
    main()
