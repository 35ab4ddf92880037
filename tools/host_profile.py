"""cProfile of the host side of the c2 training step (where the enqueue time goes).

    python tools/host_profile.py [steps]
"""
import cProfile
import pstats
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import ops  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from molclr_amd.ginet_molclr import GINet  # noqa: E402
from molclr_amd.nt_xent import NTXentLoss  # noqa: E402
from molclr_amd.optim import FusedAdam  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    batches = [(a.to(dev), b.to(dev)) for a, b in SyntheticPairBatches(512, seed=0).take(4)]
    torch.manual_seed(0)
    model = GINet(5, 300, 512).to(dev)
    opt = FusedAdam(model.parameters(), 5e-4, weight_decay=1e-5)
    crit = NTXentLoss(dev, 512, 0.1, True)

    def step(i):
        xi, xj = batches[i % len(batches)]
        for g in (xi, xj):
            g.__dict__.pop("_molclr_graph", None)
            g.__dict__.pop("_molclr_pair_graph", None)
        opt.zero_grad()
        _, z = model.forward_pair(xi, xj)   # MolCLR._step's default (paired pass)
        loss = crit.forward_pair(ops.l2_normalize(z))
        loss.backward()
        opt.step()
        return loss

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"enqueue {1e3 * (t1 - t0) / steps:.2f} ms/step, wall {1e3 * (time.perf_counter() - t0) / steps:.2f}")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(steps):
        step(i)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
