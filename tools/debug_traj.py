"""Adam-trajectory diagnostics for the 3-step training test (GPU).

For each GEMM implementation: gradient sign disagreements with the fp64 oracle
after step 0 (excluding pre-BatchNorm biases, whose exact gradient is 0), and
the loss at steps 0..2 next to the fp64 and fp32 oracle trajectories.

    python tools/debug_traj.py [gin|gcn]
"""
import copy
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from molclr_amd.nt_xent import NTXentLoss  # noqa: E402
from molclr_amd.ops import l2_normalize  # noqa: E402
from molclr_amd.optim import FusedAdam  # noqa: E402
from oracle.reference_cpu import RefGCN, RefGINet, RefNTXentLoss, ref_step_loss  # noqa: E402


def pre_bn_bias(name):
    return name.endswith("mlp.2.bias") or (name.startswith("gnns.") and name.count(".") == 2
                                            and name.endswith(".bias"))


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "gin"
    dev = torch.device("cuda", 0)
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    lib = _lib.load()
    B = 64
    torch.manual_seed(1)
    ref = (RefGINet if kind == "gin" else RefGCN)(3, 128, 512)
    state = copy.deepcopy(ref.state_dict())
    r64 = copy.deepcopy(ref).double()
    crit = RefNTXentLoss("cpu", B, 0.1, True)
    o64 = torch.optim.Adam(r64.parameters(), 5e-4, weight_decay=1e-5)
    o32 = torch.optim.Adam(ref.parameters(), 5e-4, weight_decay=1e-5)
    data = SyntheticPairBatches(B, seed=21)
    batches = [data.next() for _ in range(3)]
    l64, l32, g64 = [], [], None
    for step, (xi, xj) in enumerate(batches):
        for m, o, out in ((r64, o64, l64), (ref, o32, l32)):
            o.zero_grad()
            loss = ref_step_loss(m, crit, xi, xj)
            loss.backward()
            if step == 0 and m is r64:
                g64 = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
            o.step()
            out.append(loss.item())
    print("fp64 oracle", l64)
    print("fp32 oracle", l32, [abs(a - b) / abs(b) for a, b in zip(l32, l64)])
    for impl in (0, 1, 4):
        lib.molclr_gemm_set_impl(impl)
        mine = (GINet if kind == "gin" else GCN)(3, 128, 512)
        mine.load_state_dict(state)
        mine = mine.to(dev)
        cm = NTXentLoss(dev, B, 0.1, True)
        om = FusedAdam(mine.parameters(), 5e-4, weight_decay=1e-5)
        losses = []
        for step, (xi, xj) in enumerate(batches):
            om.zero_grad()
            _, zi = mine(xi.to(dev))
            _, zj = mine(xj.to(dev))
            loss = cm(l2_normalize(zi), l2_normalize(zj))
            loss.backward()
            if step == 0:
                for n, p in mine.named_parameters():
                    if pre_bn_bias(n):
                        continue
                    a = p.grad.detach().double().cpu()
                    b = g64[n]
                    flip = (torch.sign(a) != torch.sign(b)) & (b != 0)
                    if flip.any():
                        print(f"  impl{impl} {n}: {int(flip.sum())} sign flips, max |g64| "
                              f"{b[flip].abs().max().item():.2e} (param grad norm "
                              f"{b.norm().item():.2e}), rel err {((a - b).norm() / b.norm()).item():.2e}")
            om.step()
            losses.append(loss.item())
        print(f"impl{impl}", losses, [abs(a - b) / abs(b) for a, b in zip(losses, l64)])


if __name__ == "__main__":
    main()
