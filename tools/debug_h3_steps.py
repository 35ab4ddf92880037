"""Three-step c1 trajectory (tests/test_gpu_models.py::test_training_steps_match_oracle)
under the x6 and the h3 fp32 GEMMs: per-step loss error and step-0 gradient
errors / sign disagreements against the fp64 oracle."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import ops  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from molclr_amd.nt_xent import NTXentLoss  # noqa: E402
from molclr_amd.optim import FusedAdam  # noqa: E402
from oracle.reference_cpu import RefNTXentLoss, ref_step_loss  # noqa: E402
from tests.test_gpu_models import pair_models  # noqa: E402


def run(mode):
    ops.FP32_GEMM = mode
    dev = torch.device("cuda", 0)
    _, ref, mine = pair_models("gin", 3, 128, 512, seed=1)
    mine = mine.to(dev)
    B = 64
    crit_r = RefNTXentLoss("cpu", B, 0.1, True)
    crit_m = NTXentLoss(dev, B, 0.1, True)
    opt_r = torch.optim.Adam(ref.parameters(), 5e-4, weight_decay=1e-5)
    opt_m = FusedAdam(mine.parameters(), 5e-4, weight_decay=1e-5)
    data = SyntheticPairBatches(B, seed=21)
    for step in range(3):
        xi, xj = data.next()
        opt_r.zero_grad()
        lr = ref_step_loss(ref, crit_r, xi, xj)
        lr.backward()
        opt_m.zero_grad()
        _, zi = mine(xi.to(dev))
        _, zj = mine(xj.to(dev))
        lm = crit_m(ops.l2_normalize(zi), ops.l2_normalize(zj))
        lm.backward()
        torch.cuda.synchronize()
        print(f"{mode} step {step}: loss rel {abs(lm.item() - lr.item()) / abs(lr.item()):.2e}")
        if step == 0:
            pr = dict(ref.named_parameters())
            for name, p in mine.named_parameters():
                g, g64 = p.grad.cpu().double(), pr[name].grad
                e = ((g - g64).norm() / g64.norm().clamp_min(1e-300)).item()
                flips = int(((g.sign() != g64.sign()) & (g64.abs() > 1e-12)).sum())
                worst = ((g - g64).abs() / g64.abs().clamp_min(1e-30)).max().item()
                print(f"   {name:32s} rel {e:.2e} flips {flips:4d} worst-elem {worst:.1e} "
                      f"|g|max {g64.abs().max().item():.1e}")
        opt_r.step()
        opt_m.step()


if __name__ == "__main__":
    for m in sys.argv[1:] or ["x6", "h3"]:
        run(m)
