"""The benchmarked path at the benchmark's own size.

bench.py times CapturedTrainStep replays at c2 (GIN 5 x 300, B = 512, fp32)
and c5 (GIN 5 x 512, B = 1024, bf16) with the default capacity buckets
(node_quantum 256, edge_quantum 2048, node_slack 512: up to ~770 padding rows
per replay).  The h3 per-tensor scales and the weight-gradient split-K
partition see the padded row count, so the replay is held to the eager step
(the batch at its own size) here, step by step from the same state, over
several capacity buckets and replays on larger graphs:

* loss <= 1e-6 relative;
* the flat gradient <= 1e-5 norm-wise (bf16: 1e-4), every parameter
  <= 5e-5 (bf16: 5e-4) except the biases feeding a BatchNorm, whose exact
  gradient is 0 (rounding noise in any fp32 evaluation);
* BatchNorm running statistics <= 1e-6.

Step 0's loss is also held to the fp64 oracle (oracle/reference_cpu.py, the
restatement of models/ginet_molclr.py + utils/nt_xent.py + molclr.py:55-67):
1e-5 at c2, the bf16 model bound 1e-2 at c5 (tests/test_gpu_bf16.py)."""
import pytest
import torch

from molclr_amd.dataset import SyntheticPairBatches
from molclr_amd.ginet_molclr import GINet
from molclr_amd.graph_step import CapturedTrainStep
from molclr_amd.nt_xent import NTXentLoss
from molclr_amd.optim import FusedAdam
from oracle.reference_cpu import RefGINet, RefNTXentLoss, ref_step_loss

pytestmark = pytest.mark.gpu

# (layers, emb_dim, batch, precision, [(shape, seed, count), ...], tolerances)
CASES = {
    "c2": (5, 300, 512, "fp32", [("uniform", 0, 6), ("pubchem", 7, 2)],
           dict(grad=1e-5, param=5e-5, loss64=1e-5)),
    "c5": (5, 512, 1024, "bf16", [("pubchem", 0, 4), ("uniform", 7, 1)],
           dict(grad=1e-4, param=5e-4, loss64=1e-2)),
}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg", sorted(CASES))
def test_captured_step_at_bench_shape(dev, cfg):
    L, D, B, prec, sources, tol = CASES[cfg]
    cpu = [p for shape, seed, n in sources
           for p in SyntheticPairBatches(B, seed=seed, shape=shape).take(n)]
    batches = [(a.to(dev), b.to(dev)) for a, b in cpu]
    torch.manual_seed(0)
    model = GINet(L, D, 512, precision=prec).to(dev)
    # step 0 against the fp64 oracle, from the initial weights
    ref = RefGINet(L, D, 512).double()
    ref.load_state_dict({k: v.detach().cpu().double() if v.is_floating_point() else v.cpu()
                         for k, v in model.state_dict().items()})
    with torch.no_grad():
        loss64 = ref_step_loss(ref, RefNTXentLoss("cpu", B, 0.1, True), *cpu[0]).item()
    opt = FusedAdam(model.parameters(), 5e-4, weight_decay=1e-5)
    crit = NTXentLoss(dev, B, 0.1, True)
    step = CapturedTrainStep(model, opt, crit)  # bench.py's defaults
    assert (step.node_quantum, step.edge_quantum, step.node_slack) == (256, 2048, 512)
    step.prepare(batches)
    assert step.captures >= 3, step.buckets
    records = []
    order = batches + batches[:3]
    for i, (xi, xj) in enumerate(order):
        r = step.replay_vs_eager(xi, xj)
        records.append(r)
        if i == 0:
            assert abs(r["loss_eager"] - loss64) <= tol["loss64"] * abs(loss64), (r, loss64)
            assert abs(r["loss_replay"] - loss64) <= tol["loss64"] * abs(loss64), (r, loss64)
        assert r["loss_rel"] <= 1e-6, (i, r)
        assert r["grad_rel"] <= tol["grad"], (i, r)
        assert r["grad_rel_worst_param"][1] <= tol["param"], (i, r)
        assert r["running_stats_rel"] <= 1e-6, (i, r)
    # replays on graphs larger than the batch's own rounded size were exercised
    assert max(r["padding_rows"] for r in records) > 256, records
    print(cfg, "worst", max(r["grad_rel"] for r in records),
          max(r["grad_rel_worst_param"][1] for r in records),
          "padding", [r["padding_rows"] for r in records])
    step.close()
