"""BatchNorm backward at the c2 paired shape: molclr_batchnorm_seg_bwd against
molclr_batchnorm_seg_bwd_max (dz's row maxima / max slot), per-call time."""
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402


def timeit(fn, reps=50):
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
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    rows, D = (15300, 15256), 300
    R = sum(rows)
    z = (torch.randn(R, D, device=dev) * 2 + 0.5)
    dy = torch.randn(R, D, device=dev) * 1e-4
    gamma, beta = torch.rand(D, device=dev), torch.randn(D, device=dev)
    sr = (ctypes.c_int64 * 2)(*rows)
    ws_b = lib.molclr_batchnorm_seg_workspace_bytes(2, sr, D)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
    mean, inv = torch.empty(2, D, device=dev), torch.empty(2, D, device=dev)
    rm, rv, y = torch.zeros(D, device=dev), torch.ones(D, device=dev), torch.empty(R, D, device=dev)
    st = ops._stream(z)
    lib.molclr_batchnorm_seg_fwd(z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(),
                                 rv.data_ptr(), None, y.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                 2, sr, D, 0, 0.1, 1e-5, 1, 1, ws.data_ptr(), ws_b, st)
    dz = torch.empty(R, D, device=dev)
    dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    parts = torch.empty(lib.molclr_bn_row_parts(D), R, device=dev)
    slot = torch.zeros(2048, device=dev)
    t0 = timeit(lambda: lib.molclr_batchnorm_seg_bwd(
        dy.data_ptr(), z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
        inv.data_ptr(), dz.data_ptr(), dg.data_ptr(), db.data_ptr(), 2, sr, D, 0, 1, 1,
        ws.data_ptr(), ws_b, st))
    t1 = timeit(lambda: lib.molclr_batchnorm_seg_bwd_max(
        dy.data_ptr(), z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
        inv.data_ptr(), dz.data_ptr(), dg.data_ptr(), db.data_ptr(), 2, sr, D, 1, 1,
        parts.data_ptr(), None, ws.data_ptr(), ws_b, st))
    t2 = timeit(lambda: lib.molclr_batchnorm_seg_bwd_max(
        dy.data_ptr(), z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
        inv.data_ptr(), dz.data_ptr(), dg.data_ptr(), db.data_ptr(), 2, sr, D, 1, 1,
        parts.data_ptr(), slot.data_ptr(), ws.data_ptr(), ws_b, st))
    print(f"bn_bwd (3 kernels): plain {t0:.1f} us | row maxima {t1:.1f} us | + slot {t2:.1f} us")


if __name__ == "__main__":
    main()
