"""Ablations of the q6 x6 GEMM main loop (tools/exp/q6_abl.hip): per-launch
time with one part removed at a time, at the c2 paired shapes, next to the
product kernel (molclr_gemm_f32_bplanes_tile 9, no epilogue).

    bash tools/exp/build_q6_abl.sh && python tools/q6_abl.py [rows]
"""
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib, ops  # noqa: E402

NAMES = {0: "full copy", 1: "no A loads", 2: "no A split", 3: "no A loads+split",
         4: "no B staging", 8: "no MFMA", 16: "no epilogue", 32: "no K-step barrier",
         64: "no B LDS reads", 7: "no A, no B staging (LDS reads + MFMA)",
         68: "no B staging + no B reads", 36: "no B staging, no barrier",
         12: "no B staging, no MFMA", 24: "no MFMA, no epilogue", 72: "no MFMA, no B reads",
         39: "MFMA + B reads only (no barrier)", 103: "MFMA only",
         128: "+ the product's MASK zeroing", 256: "+ B loaded two K steps ahead",
         512: "B loads kept, LDS stores dropped", 384: "+ MASK zeroing, B two steps ahead",
         1024: "B staged by LDS-DMA", 2048: "K order rotated per block",
         3072: "LDS-DMA + K rotation", 4096: "8 waves x 32 rows share a B stage",
         5120: "8 waves + LDS-DMA"}


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
    exp = ctypes.CDLL(str(ROOT / "tools" / "exp" / "libq6_abl.so"))
    P, I = ctypes.c_void_p, ctypes.c_int64
    exp.q6_abl.argtypes = [ctypes.c_int, P, P, P, I, I, I, I, I, I, I, P]
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 30556
    st = _lib.stream_of(dev)
    torch.manual_seed(0)
    for N, K in ((600, 300), (300, 600)):
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        C = torch.empty(M, N, device=dev)
        planes = ops.weight_planes(W, N, K, K, 0)
        npad = (N + 127) // 128 * 128
        kp = (K + 31) // 32 * 32
        ws_b = lib.molclr_gemm_f32_workspace_bytes(M, N, K)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        fl = 2.0 * M * N * K
        t = timeit(lambda: lib.molclr_gemm_f32_bplanes_tile(
            A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, N, 0, 0, None, None, 0,
            ws.data_ptr(), ws_b, st, 9))
        ref = C.clone()
        print(f"M={M} N={N} K={K}: product q6 {t*1e6:6.1f} us ({fl/t/1e12:5.1f} TF)", flush=True)
        same = {}
        for abl in NAMES:
            rc = exp.q6_abl(abl, A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, kp,
                            npad, N, st)
            assert rc == 0, (abl, rc)
            torch.cuda.synchronize()
            same[abl] = torch.equal(C, ref) if abl in (0, 128, 256, 384, 1024, 4096, 5120) else None
        # rounds of all variants interleaved, median per variant (box noise ~5-10 %)
        times = {abl: [] for abl in NAMES}
        for _ in range(5):
            for abl in NAMES:
                times[abl].append(timeit(lambda: exp.q6_abl(
                    abl, A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K, kp, npad, N,
                    st), reps=10))
        for abl, name in NAMES.items():
            t = sorted(times[abl])[2]
            print(f"  abl {abl:3d} {name:40s} {t*1e6:6.1f} us"
                  + ("" if same[abl] is None else f"  (bit-identical to product: {same[abl]})"),
                  flush=True)


if __name__ == "__main__":
    main()
