"""q6 vs p6 vs fp64 on the accuracy-test shape; per-column-block error profile."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
M, N, K = 1000, 600, 300
torch.manual_seed(K)
Am = torch.randn(M, K, dtype=torch.float64) * torch.logspace(-3, 3, K).double()
Bm = torch.randn(K, N, dtype=torch.float64)
A = Am.contiguous().float()
Bt = Bm.t().contiguous().float()
ref = A.double() @ Bt.double().t()
for t in (5, 7, 9):
    lib.molclr_gemm_bplanes_set_impl(t)
    out = ops.gemm_w(A.to(dev), Bt.to(dev), M, N, K, K, K, 0, 0).double().cpu()
    err = out - ref
    print(t, "rel", (err.norm() / ref.norm()).item(), "max", err.abs().max().item())
    colblk = [(err[:, c:c + 32].norm() / ref[:, c:c + 32].norm()).item() for c in range(0, N, 32)]
    rowblk = [(err[r:r + 32].norm() / ref[r:r + 32].norm()).item() for r in range(0, M, 32)]
    print("  col blocks", " ".join(f"{v:.1e}" for v in colblk))
    print("  row blocks", " ".join(f"{v:.1e}" for v in rowblk[:16]))
# exact-integer check: small ints, any reordering exact
Ai = torch.randint(-3, 4, (M, K)).float()
Bi = torch.randint(-3, 4, (N, K)).float()
refi = Ai.double() @ Bi.double().t()
for t in (5, 9):
    lib.molclr_gemm_bplanes_set_impl(t)
    out = ops.gemm_w(Ai.to(dev), Bi.to(dev), M, N, K, K, K, 0, 0).double().cpu()
    print(t, "int max err", (out - refi).abs().max().item())
