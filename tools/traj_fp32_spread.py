"""How far the reference's OWN fp32 path drifts from fp64 over the 3-step c1
trajectory of tests/test_gpu_models.py::test_training_steps_match_oracle
(same seeds, same batches, Adam lr 5e-4 / wd 1e-5): the per-step loss and the
parameter spread of the fp32 oracle (torch CPU fp32 -- what the reference
computes) and of the same oracle with every Linear's product summed in the
opposite row order (another legitimate fp32 order), each against fp64.

CPU only: python tools/traj_fp32_spread.py [--write-golden]
  --write-golden: also writes tests/golden/traj_fp32_spread.json (per step and
  per parameter, the larger of the two fp32 variants' spreads), which bounds
  the GPU trajectory test.
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


def pre_bn_bias(name: str) -> bool:
    """tests/test_gpu_models.py's exemption: biases that a BatchNorm follows."""
    return name.endswith("mlp.2.bias") or (name.startswith("gnns.") and name.count(".") == 2
                                            and name.endswith(".bias"))


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
    golden = {"loss_rel_per_step": [0.0, 0.0, 0.0], "param_rel": {}}
    for name, m in variants.items():
        ls = run(m)
        drift = max((p.detach().double() - p64[n].detach()).abs().max().item()
                    for n, p in m.named_parameters())
        # the test's norm-wise relative check, pre-BatchNorm biases excluded
        rels = {n: ((p.detach().double() - p64[n].detach()).norm()
                    / p64[n].detach().norm().clamp_min(1e-30)).item()
                for n, p in m.named_parameters() if not pre_bn_bias(n)}
        worst = sorted(rels.items(), key=lambda kv: -kv[1])[:3]
        golden["loss_rel_per_step"] = [max(g, abs(a - b) / abs(b))
                                       for g, a, b in zip(golden["loss_rel_per_step"], ls, l64)]
        for n, r in rels.items():
            golden["param_rel"][n] = max(golden["param_rel"].get(n, 0.0), r)
        print(json.dumps({"variant": name,
                          "loss_rel_err_per_step": [abs(a - b) / abs(b) for a, b in zip(ls, l64)],
                          "param_max_abs_diff_after_3": drift,
                          "param_rel_worst_after_3": worst}))
    if "--write-golden" in sys.argv:
        out = ROOT / "tests" / "golden" / "traj_fp32_spread.json"
        out.write_text(json.dumps(golden, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
