"""How far the reference's OWN fp32 path drifts from fp64 over the 3-step c1
trajectory of tests/test_gpu_models.py::test_training_steps_match_oracle
(same seeds, same batches, Adam lr 5e-4 / wd 1e-5): the per-step loss and the
parameter spread of the fp32 oracle (torch CPU fp32 -- what the reference
computes) and of the same oracle with every Linear's product summed in the
opposite row order (another legitimate fp32 order), each against fp64.

CPU only: python tools/traj_fp32_spread.py
"""
import copy
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from oracle.reference_cpu import RefGINet, RefNTXentLoss, ref_step_loss  # noqa: E402


class _RevLinear(torch.autograd.Function):
    """x W^T + b with the K sum in reverse order (fp32): a different but
    equally valid rounding of the same product."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        return x.flip(1) @ W.flip(1).T + b

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        return g @ W, g.T @ x, g.sum(0)


def rev_linears(model):
    for m in model.modules():
        if isinstance(m, torch.nn.Linear):
            m.forward = (lambda mod: (lambda x: _RevLinear.apply(x, mod.weight, mod.bias)))(m)
    return model


def run(model, steps=3, B=64):
    crit = RefNTXentLoss("cpu", B, 0.1, True)
    opt = torch.optim.Adam(model.parameters(), 5e-4, weight_decay=1e-5)
    data = SyntheticPairBatches(B, seed=21)
    losses = []
    for _ in range(steps):
        xi, xj = data.next()
        opt.zero_grad()
        loss = ref_step_loss(model, crit, xi, xj)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


def main():
    torch.manual_seed(1)
    ref = RefGINet(3, 128, 512)
    r64 = copy.deepcopy(ref).double()
    variants = {"fp32 (reference)": copy.deepcopy(ref), "fp32 reversed K": rev_linears(copy.deepcopy(ref))}
    l64 = run(r64)
    p64 = dict(r64.named_parameters())
    for name, m in variants.items():
        ls = run(m)
        drift = max((p.detach().double() - p64[n].detach()).abs().max().item()
                    for n, p in m.named_parameters())
        print(json.dumps({"variant": name,
                          "loss_rel_err_per_step": [abs(a - b) / abs(b) for a, b in zip(ls, l64)],
                          "param_max_abs_diff_after_3": drift}))


if __name__ == "__main__":
    main()
