"""Small fp32 GEMMs of the readout heads (2B = 1024 rows at c2): torch.mm
(rocBLAS / hipBLASLt fp32) against the library's x6 products, HIP events."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from molclr_amd import ops  # noqa: E402


def t(fn, reps=200):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


dev = torch.device("cuda")
torch.backends.cuda.matmul.allow_tf32 = False
M = 1024
for K, N in ((300, 512), (512, 512), (512, 256)):
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    b = torch.randn(N, device=dev)
    dy = torch.randn(M, N, device=dev)
    ref = (x.double() @ W.double().T + b.double())
    y1 = torch.addmm(b, x, W.T)
    y2 = ops.linear_fwd(x, W, b)
    e1 = ((y1.double() - ref).norm() / ref.norm()).item()
    e2 = ((y2.double() - ref).norm() / ref.norm()).item()
    tf = t(lambda: torch.addmm(b, x, W.T))
    tl = t(lambda: ops.linear_fwd(x, W, b))
    tw = t(lambda: dy.T @ x)
    tlw = t(lambda: ops.linear_bwd(dy, x, W, need_x=False))
    tdx = t(lambda: dy @ W)
    tldx = t(lambda: ops.linear_bwd(dy, x, W, need_w=False, need_b=False))
    print(f"{M}x{K}->{N}: fwd torch {tf:.1f} us (err {e1:.1e}) lib {tl:.1f} us (err {e2:.1e}); "
          f"wgrad torch {tw:.1f} lib {tlw:.1f}; dgrad torch {tdx:.1f} lib {tldx:.1f}")
