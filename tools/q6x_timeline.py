"""Phase timeline of the ping-pong q6 kernel (tools/exp/q6x.hip, ABL 32):
s_memtime stamps at every phase boundary of every wave; prints the median
cycles per phase part for each wave group, lin1 (x6) and dz1 (h3) shapes.

    bash tools/exp/build_q6x.sh && python tools/q6x_timeline.py [variant]
"""
import ctypes
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS_RELU, EPI_NONE  # noqa: E402


def main():
    variant = int(sys.argv[1]) if len(sys.argv) > 1 else 132
    dev = torch.device("cuda", 0)
    exp = ctypes.CDLL(str(ROOT / "tools" / "exp" / "libq6x.so"))
    P, I, Ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    exp.q6x.argtypes = [Ci, Ci, Ci, P, P, P, I, I, I, I, I, I, I, P, P, I, P, P, P, P, P, Ci, P, P,
                        I, P]
    st = _lib.stream_of(dev)
    torch.manual_seed(0)
    M = 30556
    for name, N, K, epi in (("lin1 x6", 600, 300, EPI_BIAS_RELU), ("lin2 x6", 300, 600, EPI_NONE)):
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        planes = ops.weight_planes(W, N, K, K, 0, "x6")
        npad, kp = (N + 127) // 128 * 128, (K + 31) // 32 * 32
        C = torch.empty(M, N, device=dev)
        blocks = ((M + 255) // 256) * ((N + 159) // 160)
        stamps = torch.zeros(blocks * 8 * 64, dtype=torch.int64, device=dev)
        for _ in range(3):
            rc = exp.q6x(variant, epi, 0, A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K, K,
                         kp, npad, N, b.data_ptr(), None, 0, None, None, None, None, None, 0,
                         stamps.data_ptr(), None, M, st)
            assert rc == 0, rc
        torch.cuda.synchronize()
        t = stamps.view(blocks, 8, 64).cpu()
        S = kp // 32
        # group 0: [pre, (comp, wait, bar, load, bar) x (S-1), comp, epi, end]
        # group 1: [pre, stagger, (comp, wait, bar, load, bar) x (S-1), comp, epi, end]
        parts = {g: {k: [] for k in ("compute", "vmwait", "barrier1", "load", "barrier2", "epilogue",
                                      "block")} for g in (0, 1)}
        for blk in range(blocks):
            for w in range(8):
                g = w // 4
                s = t[blk, w].tolist()
                base = 1 if g == 0 else 2
                for i in range(S - 1):
                    j = base + 5 * i
                    prev = s[j - 1]
                    parts[g]["compute"].append(s[j] - prev)
                    parts[g]["vmwait"].append(s[j + 1] - s[j])
                    parts[g]["barrier1"].append(s[j + 2] - s[j + 1])
                    parts[g]["load"].append(s[j + 3] - s[j + 2])
                    parts[g]["barrier2"].append(s[j + 4] - s[j + 3])
                last = base + 5 * (S - 1)
                parts[g]["epilogue"].append(s[last + 2] - s[last + 1])
                parts[g]["block"].append(s[last + 2] - s[0])
        print(f"{name}: S={S} steps, {blocks} blocks; median cycles (s_memtime ticks)")
        for g in (0, 1):
            print(f"  group {g}: " + ", ".join(f"{k} {statistics.median(v):.0f}"
                                             for k, v in parts[g].items()), flush=True)


if __name__ == "__main__":
    main()
