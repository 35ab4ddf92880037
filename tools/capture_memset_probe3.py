"""Which captured zeroing is reliable?  Regions poisoned (3e38) before every
replay; after the replay (and a device synchronize) they must read zero:

  leaf   -- hipMemsetAsync through the library (molclr_absmax_f32 with no
            rows: memset of its 8 KB slot and nothing else), nothing after it
  read   -- the same memset, then a kernel that copies the region elsewhere
            (the copy must be zero too)
  kernel -- torch's zero_() (a fill kernel), nothing after it
  copy   -- torch's copy_() between two device tensors (a D2D memcpy), the
            destination must equal the source

    python tools/capture_memset_probe3.py [replays]
"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    x = torch.randn(16, device=dev)
    src = torch.zeros(2048, device=dev)
    for case in ("leaf", "read", "kernel", "copy"):
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
            b = torch.empty(2048, device=dev)
            st = torch.cuda.current_stream().cuda_stream
            y = x * 2
            if case == "kernel":
                b.zero_()
            elif case == "copy":
                b.copy_(src)
            else:
                assert lib.molclr_absmax_f32(y.data_ptr(), 0, 0, 1, b.data_ptr(), 0, st) == 0
            c = b * 1.0 if case == "read" else None
        bad_b = bad_c = 0
        for r in range(reps):
            b.fill_(3e38)
            if c is not None:
                c.fill_(3e38)
            g.replay()
            torch.cuda.synchronize()
            bad_b += int(bool((b != 0).any().item()))
            if c is not None:
                bad_c += int(bool((c != 0).any().item()))
        print(f"{case:7s}: region nonzero after {bad_b} of {reps} replays"
              + (f", its copy nonzero after {bad_c}" if c is not None else ""), flush=True)


if __name__ == "__main__":
    main()
