"""Ablations of the w6 weight-gradient main loop (tools/exp/w6_abl.hip, h3
form): per-launch time with one part removed at a time, at the c2 shapes,
next to the product kernel (molclr_linear_wgrad_h3 without bias sums is not
exposed; the product line is the full copy, variant 0).

    bash tools/exp/build_w6_abl.sh && python tools/w6_abl.py [rows]
"""
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent

NAMES = {0: "full copy", 1: "no global loads", 2: "no split + LDS stores",
         4: "no MFMA", 8: "no fragment reads", 16: "no barriers",
         3: "no loads, no split (reads + MFMA)", 12: "no reads, no MFMA (loads + split)",
         6: "no split, no MFMA (loads + reads)", 5: "no loads, no MFMA (split + reads)",
         32: "loads two phases ahead (LDS-DMA slot)", 48: "DMA slot, no barriers"}


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
    exp = ctypes.CDLL(str(ROOT / "tools" / "exp" / "libw6_abl.so"))
    P, I = ctypes.c_void_p, ctypes.c_int64
    exp.w6_abl.argtypes = [ctypes.c_int, P, P, P, I, I, I, ctypes.c_int, ctypes.c_int, P]
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 30556
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    torch.manual_seed(0)
    for M, N in ((600, 300), (300, 600)):
        A = torch.randn(K, M, device=dev)
        B = torch.randn(K, N, device=dev)
        ntiles = ((M + 127) // 128) * ((N + 159) // 160)
        nk = (K + 31) // 32
        s = max(1, min(256 // ntiles, nk // 8))
        kps = (nk + s - 1) // s
        splits = (nk + kps - 1) // kps
        part = torch.zeros(2 * splits, M, N, device=dev)
        ref = (A.double().t() @ B.double())
        fl = 2.0 * M * N * K
        res = {}
        for abl in NAMES:
            part.zero_()
            rc = exp.w6_abl(abl, A.data_ptr(), B.data_ptr(), part.data_ptr(), M, N, K, kps, splits, st)
            assert rc == 0, (abl, rc)
            torch.cuda.synchronize()
            if abl in (0, 32):
                res[abl] = part.clone()
        same = torch.equal(res[0], res[32])
        err = ((res[0].double().sum(0) - ref).norm() / ref.norm()).item()
        print(f"M={M} N={N} K={K} splits={splits} x {kps} K tiles: full copy err {err:.2e}, "
              f"DMA variant bit-identical {same}", flush=True)
        times = {abl: [] for abl in NAMES}
        for _ in range(5):
            for abl in NAMES:
                times[abl].append(timeit(lambda: exp.w6_abl(
                    abl, A.data_ptr(), B.data_ptr(), part.data_ptr(), M, N, K, kps, splits, st),
                    reps=10))
        for abl, name in NAMES.items():
            t = sorted(times[abl])[2]
            print(f"  abl {abl:3d} {name:42s} {t*1e6:6.1f} us ({fl/t/1e12:5.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
