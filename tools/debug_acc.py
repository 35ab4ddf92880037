"""Replicates test_gemm_split_bf16_accuracy and prints every impl's error."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()


def rel(a, b):
    a = a.double().cpu()
    return ((a - b).norm() / b.norm()).item()


for ak, bk in ((0, 0), (0, 1)):
    for M, N, K, positive in ((1000, 600, 300, False), (300, 600, 15700, False),
                              (1000, 600, 300, True), (300, 600, 15700, True)):
        torch.manual_seed(K)
        if positive:
            Am = torch.rand(M, K, dtype=torch.float64)
            Bm = torch.rand(K, N, dtype=torch.float64)
        else:
            Am = torch.randn(M, K, dtype=torch.float64) * torch.logspace(-3, 3, K).double()
            Bm = torch.randn(K, N, dtype=torch.float64)
        A = (Am.t() if ak else Am).contiguous().float()
        Bt = (Bm if bk else Bm.t()).contiguous().float()
        ref = (A.double().t() if ak else A.double()) @ (Bt.double() if bk else Bt.double().t())
        res = {}
        for impl in (0, 1, 5, 6, "bp0", "bp9"):
            if isinstance(impl, str):
                lib.molclr_gemm_bplanes_set_impl(int(impl[2:]))
                out = ops.gemm_w(A.to(dev), Bt.to(dev), M, N, K, M if ak else K, N if bk else K, ak, bk)
                lib.molclr_gemm_bplanes_set_impl(0)
            else:
                lib.molclr_gemm_set_impl(impl)
                out = ops.gemm(A.to(dev), Bt.to(dev), M, N, K, M if ak else K, N if bk else K, ak, bk)
                lib.molclr_gemm_set_impl(5)
            res[impl] = rel(out, ref)
        print(ak, bk, M, N, K, positive, " ".join(f"{k}:{v:.2e}" for k, v in res.items()), flush=True)
