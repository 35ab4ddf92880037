"""Data-parallel NT-Xent on the GPU (BASELINE config c4).

* c4 as W = 8 simulated ranks through the C ABI: every rank owns its rows
  [zj_local; zi_local] (2 x 512) and sees the gathered columns (8192 x 256)
  and gathered logsumexp -- molclr_ntxent_fwd / _bwd with nrows != ncols and
  the global row offsets of molclr_amd.distributed.global_row_index.  The
  assembled loss and gradients must equal the single-process NT-Xent of the
  global batch 4096 (utils/nt_xent.py:47-65; oracle/ntxent_math in float64,
  itself pinned by the reference's goldens) at 1e-5 norm-wise.
* The product's ``group=`` branch (ops._NTXent: gather_rows / gather_lse /
  loss all-reduce, the gradient all-reduce) under RCCL with world size 1: the
  collectives run for real and the result is bit-identical to the
  single-process path.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch

from molclr_amd import _lib
from molclr_amd import distributed as mdist
from oracle import ntxent_math

pytestmark = pytest.mark.gpu
TOL = 1e-5


def rel(a, b):
    a = np.asarray(torch.as_tensor(a).detach().double().cpu())
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _prep(lib, R, cosine, dev):
    n, C = R.shape
    rh = torch.empty_like(R)
    nrm = torch.empty(n, device=dev)
    assert lib.molclr_ntxent_prep(R.data_ptr(), rh.data_ptr(), nrm.data_ptr(), n, C, int(cosine),
                                  None) == 0
    return rh, nrm


@pytest.mark.parametrize("W,Bl,C,cosine,impl", [(8, 512, 256, True, 0), (8, 512, 256, True, 1),
                                                (8, 512, 256, True, 2), (8, 512, 256, True, 3),
                                                (8, 512, 256, True, -1), (2, 512, 256, False, 2),
                                                (2, 512, 256, False, 3), (3, 37, 64, False, 0),
                                                (3, 36, 64, False, 1), (3, 37, 64, False, -1)])
def test_row_sharded_ntxent_simulated_ranks(dev, W, Bl, C, cosine, impl):
    """impl: 0 fused kernels, 1 x6 GEMM formulation, 2 h3 transposed GEMM
    formulation (S^T by the h3 GEMM, dR by the h3 weight-gradient product),
    -1 automatic."""
    lib = _lib.load()
    B = W * Bl
    T = 0.1
    rng = np.random.default_rng(W * Bl)
    zi = rng.standard_normal((B, C)).astype(np.float32)
    zj = (0.5 * zi + rng.standard_normal((B, C))).astype(np.float32)
    if not cosine:  # dot similarity needs tame logits: unit rows, as after F.normalize
        zi /= np.linalg.norm(zi, axis=1, keepdims=True)
        zj /= np.linalg.norm(zj, axis=1, keepdims=True)
    loss_ref, dzi_ref, dzj_ref = ntxent_math.ntxent(zi, zj, T, cosine)
    zid, zjd = torch.from_numpy(zi).to(dev), torch.from_numpy(zj).to(dev)
    # each rank: local rows, prep (row scaling), then what gather_rows returns
    ranks = []
    for r in range(W):
        sl = slice(r * Bl, (r + 1) * Bl)
        rows, nrm = _prep(lib, torch.cat([zjd[sl], zid[sl]]).contiguous(), cosine, dev)
        ranks.append((rows, nrm, mdist.global_row_index(Bl, r, W, dev)))
    g = torch.stack([rk[0] for rk in ranks])                  # all_gather stack
    cols = torch.cat([g[:, :Bl].reshape(B, C), g[:, Bl:].reshape(B, C)]).contiguous()
    ws_bytes = lib.molclr_ntxent_workspace_bytes(2 * Bl, 2 * B, C)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    # formulation 1 keeps S from the forward for rank 0's backward (the others
    # recompute it): both paths are checked
    sim_bytes = lib.molclr_ntxent_sim_bytes(2 * Bl, 2 * B, C, impl)
    sims = [torch.empty(max(sim_bytes, 4), dtype=torch.uint8, device=dev) if r == 0 and sim_bytes
            else None for r in range(W)]
    lses, loss = [], 0.0
    for (rows, _, gidx), sim in zip(ranks, sims):
        lse = torch.empty(2 * Bl, device=dev)
        lr = torch.empty(2 * Bl, device=dev)
        assert lib.molclr_ntxent_fwd_impl(rows.data_ptr(), gidx.data_ptr(), cols.data_ptr(),
                                          2 * Bl, 2 * B, C, B, T, lse.data_ptr(), lr.data_ptr(),
                                          _lib.ptr(sim), ws.data_ptr(), ws_bytes, None,
                                          impl) == 0
        lses.append(lse)
        loss += lr.double().sum().item()
    lg = torch.stack(lses)
    lse_cols = torch.cat([lg[:, :Bl].reshape(-1), lg[:, Bl:].reshape(-1)]).contiguous()
    gl = torch.ones((), device=dev)
    dzi, dzj = [], []
    for (rows, nrm, gidx), sim in zip(ranks, sims):
        drh = torch.empty_like(rows)
        assert lib.molclr_ntxent_bwd_impl(rows.data_ptr(), gidx.data_ptr(), cols.data_ptr(),
                                          lse_cols.data_ptr(), gl.data_ptr(), 2 * Bl, 2 * B, C, B,
                                          T, _lib.ptr(sim), drh.data_ptr(), ws.data_ptr(),
                                          ws_bytes, None, impl) == 0
        dR = torch.empty_like(rows)
        assert lib.molclr_ntxent_prep_bwd(drh.data_ptr(), rows.data_ptr(), nrm.data_ptr(),
                                          dR.data_ptr(), 2 * Bl, C, int(cosine), None) == 0
        dzj.append(dR[:Bl])
        dzi.append(dR[Bl:])
    torch.cuda.synchronize()
    assert abs(loss - loss_ref) <= TOL * abs(loss_ref), (loss, loss_ref)
    assert rel(torch.cat(dzi), dzi_ref) < TOL
    assert rel(torch.cat(dzj), dzj_ref) < TOL


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture()
def rccl_world1(dev):
    import torch.distributed as dist
    assert not dist.is_initialized()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield dist.group.WORLD
    dist.destroy_process_group()


def test_ntxent_group_branch_rccl_world1(dev, rccl_world1):
    """ops._NTXent's group branch and the gradient all-reduce with real RCCL
    collectives (world size 1): bit-identical to the single-process path."""
    from molclr_amd.nt_xent import NTXentLoss
    torch.manual_seed(0)
    B, C = 512, 256
    zi = torch.randn(B, C, device=dev)
    zj = zi + 0.8 * torch.randn(B, C, device=dev)
    outs = []
    for group in (None, rccl_world1):
        a = zi.clone().requires_grad_(True)
        b = zj.clone().requires_grad_(True)
        loss = NTXentLoss(dev, B, 0.1, True, group=group)(a, b)
        loss.backward()
        outs.append((loss.detach(), a.grad, b.grad))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    flat = torch.arange(8, dtype=torch.float32, device=dev)
    mdist.allreduce_grads(flat)
    assert torch.equal(flat, torch.arange(8, dtype=torch.float32, device=dev))
    rows = torch.randn(2 * 4, 3, device=dev)
    assert torch.equal(mdist.gather_rows(rows), rows)          # world 1: identity order
    assert torch.equal(mdist.gather_lse(rows[:, 0].contiguous()), rows[:, 0])


def test_training_step_under_rccl_world1(dev, rccl_world1):
    """A product training step through the data-parallel code path (group NT-Xent,
    gradient all-reduce, parameter broadcast) equals the single-process step."""
    import copy

    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.ginet_molclr import GINet
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    from molclr_amd.optim import FusedAdam
    torch.manual_seed(3)
    m0 = GINet(2, 64, 128).to(dev)
    m1 = copy.deepcopy(m0)
    xi, xj = SyntheticPairBatches(32, seed=9).next()
    xi, xj = xi.to(dev), xj.to(dev)
    res = []
    for m, group in ((m0, None), (m1, rccl_world1)):
        opt = FusedAdam(m.parameters(), 5e-4, weight_decay=1e-5)
        mdist.broadcast_params(opt.flat)
        opt.zero_grad()
        loss = NTXentLoss(dev, 32, 0.1, True, group=group)(l2_normalize(m(xi)[1]),
                                                            l2_normalize(m(xj)[1]))
        loss.backward()
        if group is not None:
            mdist.allreduce_grads(opt.flat_grad)
        opt.step()
        res.append(opt.flat.clone())
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_overlapped_reducer_step_rccl_world1(dev, rccl_world1, kind):
    """The paired-view training step with the bucketed, overlapped gradient
    all-reduce (executor done-events, side-stream RCCL buckets) under real
    RCCL (world size 1): parameters after the step bit-identical to the
    single-process step."""
    import copy

    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    from molclr_amd.optim import FusedAdam
    torch.manual_seed(4)
    m0 = (GINet if kind == "gin" else GCN)(3, 64, 128).to(dev)
    m1 = copy.deepcopy(m0)
    xi, xj = SyntheticPairBatches(32, seed=12).next()
    xi, xj = xi.to(dev), xj.to(dev)
    out = []
    for m, group in ((m0, None), (m1, rccl_world1)):
        params = mdist.bucketed_parameters(m) if group is not None else m.parameters()
        opt = FusedAdam(params, 5e-4, weight_decay=1e-5)
        red = mdist.OverlappedGradReducer(m, opt, group) if group is not None else None
        for _ in range(2):
            opt.zero_grad()
            if red is not None:
                red.arm()
            _, z = m.forward_pair(xi, xj)
            loss = NTXentLoss(dev, 32, 0.1, True, group=group).forward_pair(l2_normalize(z))
            loss.backward()
            if red is not None:
                assert red.calls == 1  # the executor drove the buckets
                red.finish()
            opt.step()
        out.append({n: p.detach().clone() for n, p in m.named_parameters()})
    for n in out[0]:
        assert torch.equal(out[0][n], out[1][n]), n


def _param_report(model, opt_a, opt_b, names=("a", "b")):
    """Per-parameter rel error of opt_a.flat_grad against opt_b.flat_grad with
    both norms (which side is wrong), worst first."""
    name_of = {id(p): n for n, p in model.named_parameters()}
    rows = []
    for (p, off, n) in opt_a.views:  # same bucketed layout on both sides
        ga = opt_a.flat_grad[off:off + n].double()
        gb = opt_b.flat_grad[off:off + n].double()
        nb = gb.norm().item()
        rows.append((((ga - gb).norm().item() / max(nb, 1e-30)), name_of.get(id(p), "?"),
                     ga.norm().item(), nb))
    rows.sort(reverse=True)
    return "; ".join(f"{nm}: rel {r:.3g} |{names[0]}| {na:.4g} |{names[1]}| {nb:.4g}"
                     for r, nm, na, nb in rows[:8])


def _snapshot_buffers(opt, model):
    """Pinned host buffers for _snapshot (allocated once, outside the loop)."""
    ts = [opt.flat, opt.exp_avg, opt.exp_avg_sq, opt._step_dev]
    for bn in model.batch_norms:
        ts += [bn.running_mean, bn.running_var, bn.num_batches_tracked]
    return [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in ts]


def _snapshot(opt, model, bufs):
    """Asynchronous host copies (no device allocation and no synchronisation:
    the failure this test guards against depended on both)."""
    ts = [opt.flat, opt.exp_avg, opt.exp_avg_sq, opt._step_dev]
    for bn in model.batch_norms:
        ts += [bn.running_mean, bn.running_var, bn.num_batches_tracked]
    for b, t in zip(bufs, ts):
        b.copy_(t, non_blocking=True)
    return bufs


def _restore(opt, model, bufs):
    ts = [opt.flat, opt.exp_avg, opt.exp_avg_sq, opt._step_dev]
    for bn in model.batch_norms:
        ts += [bn.running_mean, bn.running_var, bn.num_batches_tracked]
    with torch.no_grad():
        for t, b in zip(ts, bufs):
            t.copy_(b)


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_captured_dp_step_rccl_world1(dev, rccl_world1, kind):
    """The data-parallel step captured as HIP graphs (CapturedTrainStep with
    the group NT-Xent's all-gathers and the overlapped bucket all-reduces
    inside the graph) against the eager data-parallel step under real RCCL
    (world size 1), step by step from the same state over several capacity
    buckets: loss to 1e-6, gradients to 5e-5 norm-wise (the padded rows only
    change the weight gradients' split-K partition, i.e. the fp32 summation
    order of dW over ~2k rows: measured 2.3e-5 at this B = 32 size, against
    ~1e-3 for the reference's own fp32 vs fp64).  On a mismatch the message
    names every step's capture / replay, the worst parameters with both
    sides' norms, and a third (eager, no process group) gradient from the
    same state, so the failing side is identified."""
    _captured_dp_case(dev, rccl_world1, kind)


def _captured_dp_case(dev, group, kind, seed=6, n_pairs=5, min_captures=2):
    import copy

    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    from molclr_amd.graph_step import CapturedTrainStep
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import bump_param_generation, l2_normalize
    from molclr_amd.optim import FusedAdam
    torch.manual_seed(seed)
    ref = (GINet if kind == "gin" else GCN)(3, 64, 128).to(dev)
    cap = copy.deepcopy(ref)
    B = 32
    pairs = [tuple(b.to(dev) for b in p) for p in SyntheticPairBatches(B, seed=31).take(n_pairs)]
    opts, reds = [], []
    for m in (ref, cap):
        opt = FusedAdam(mdist.bucketed_parameters(m), 5e-4, weight_decay=1e-5)
        mdist.broadcast_params(opt.flat)
        opts.append(opt)
        reds.append(mdist.OverlappedGradReducer(m, opt, group))
    crit = NTXentLoss(dev, B, 0.1, True, group=group)
    step = CapturedTrainStep(cap, opts[1], crit, node_quantum=128, edge_quantum=512, node_slack=0,
                             reducer=reds[1])

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    history = []
    bufs = _snapshot_buffers(opts[0], ref)
    try:
        for i, (xi, xj) in enumerate(pairs + pairs[:2]):
            with torch.no_grad():  # ref := cap's state
                for a, b in ((opts[0].flat, opts[1].flat), (opts[0].exp_avg, opts[1].exp_avg),
                             (opts[0].exp_avg_sq, opts[1].exp_avg_sq),
                             (opts[0]._step_dev, opts[1]._step_dev)):
                    a.copy_(b)
                for br, bc in zip(ref.batch_norms, cap.batch_norms):
                    br.running_mean.copy_(bc.running_mean)
                    br.running_var.copy_(bc.running_var)
                    br.num_batches_tracked.copy_(bc.num_batches_tracked)
            snap = _snapshot(opts[0], ref, bufs)
            bump_param_generation()
            opts[0].zero_grad()
            reds[0].arm()
            _, z = ref.forward_pair(xi, xj)
            le = crit.forward_pair(l2_normalize(z))
            le.backward()
            reds[0].finish()
            opts[0].step()
            before = step.captures
            lc = step(xi, xj).clone()
            torch.cuda.synchronize()
            history.append("capture" if step.captures > before else "replay")
            assert abs(lc.item() - le.item()) <= 1e-6 * abs(le.item()), (i, lc.item(), le.item())
            r = rel(opts[1].flat_grad, opts[0].flat_grad)
            if r >= 5e-5:
                eager_grad = opts[0].flat_grad.clone()
                # a third gradient from the same state: eager, no group, no reducer
                _restore(opts[0], ref, snap)
                bump_param_generation()
                opts[0].zero_grad()
                _, z = ref.forward_pair(xi, xj)
                NTXentLoss(dev, B, 0.1, True).forward_pair(l2_normalize(z)).backward()
                torch.cuda.synchronize()
                third = opts[0].flat_grad.clone()
                opts[0].flat_grad.copy_(eager_grad)
                # the same replay again from the same state: persistent damage
                # to the graph's own state, or a transient race?
                _restore(opts[1], cap, snap)
                bump_param_generation()
                step(xi, xj)
                torch.cuda.synchronize()
                again = rel(opts[1].flat_grad, eager_grad)
                msg = (f"step {i} ({history}): again {again:.3g}; rel(captured, eager DP) = {r:.3g}; "
                       f"rel(eager DP, eager local) = {rel(eager_grad, third):.3g}; "
                       f"rel(captured, eager local) = {rel(opts[1].flat_grad, third):.3g}; "
                       f"captured vs eager DP: {_param_report(cap, opts[1], opts[0], ('cap', 'eager'))}")
                raise AssertionError(msg)
        assert step.captures >= min_captures and step.replays == len(pairs) + 2
    finally:
        step.close()  # before the fixture destroys the process group


def _churn(dev, kind, seed):
    """Create, step (eager, then captured over two buckets) and drop a model,
    leaving what such a model leaves in the process: cached weight images of
    dead weights, freed graph pools, collected autograd state."""
    import gc

    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    from molclr_amd.graph_step import CapturedTrainStep
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import l2_normalize
    from molclr_amd.optim import FusedAdam
    torch.manual_seed(seed)
    m = (GINet if kind == "gin" else GCN)(3, 64, 128).to(dev)
    opt = FusedAdam(m.parameters(), 5e-4, weight_decay=1e-5)
    crit = NTXentLoss(dev, 32, 0.1, True)
    pairs = [tuple(b.to(dev) for b in p) for p in SyntheticPairBatches(32, seed=seed).take(3)]
    for xi, xj in pairs[:2]:
        opt.zero_grad()
        _, z = m.forward_pair(xi, xj)
        crit.forward_pair(l2_normalize(z)).backward()
        opt.step()
    step = CapturedTrainStep(m, opt, crit, node_quantum=128, edge_quantum=512, node_slack=0)
    for xi, xj in pairs + pairs[:1]:
        step(xi, xj)
    torch.cuda.synchronize()
    del step, m, opt, crit, pairs
    gc.collect()


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_captured_dp_step_after_other_models(dev, rccl_world1, kind):
    """The captured data-parallel step in a process where other models were
    built, stepped eagerly and as HIP graphs, and dropped first -- the state the
    round-4 driver run left before its one failure of
    test_captured_dp_step_rccl_world1 (MLP weight gradients of the captured
    side exactly zero).  Then the same case twice more with fresh models, each
    after more churn, all against the eager data-parallel step."""
    for rep in range(3):
        _churn(dev, "gin", 100 + rep)
        _churn(dev, "gcn", 200 + rep)
        # 8 pairs: three capacity buckets (1792, 1920, 2048 nodes)
        _captured_dp_case(dev, rccl_world1, kind, seed=7 + rep, n_pairs=8, min_captures=3)


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_captured_dp_multi_rank_paths_world1(dev, rccl_world1, monkeypatch, kind):
    """The code a multi-rank run takes, reached on one GPU by
    forcing CapturedTrainStep._multi_rank() true under a real RCCL group of
    one: prepare() goes through prepare_sizes and the _global_sizes
    all-gathers; a batch no captured graph holds takes the lockstep eager
    path (CapturedTrainStep._eager: the same collectives as a replay, no
    capture); replays and eager steps alternate.  Every step is held to the
    eager data-parallel step from the same state (loss 1e-6, gradients 5e-5,
    running statistics 1e-6), and the counters say which path ran."""
    import copy

    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    from molclr_amd.graph_step import CapturedTrainStep
    from molclr_amd.nt_xent import NTXentLoss
    from molclr_amd.ops import bump_param_generation, l2_normalize
    from molclr_amd.optim import FusedAdam
    monkeypatch.setattr(CapturedTrainStep, "_multi_rank", lambda self: True)
    calls = []
    real_gs = CapturedTrainStep._global_sizes
    monkeypatch.setattr(CapturedTrainStep, "_global_sizes",
                        lambda self, sizes: calls.append(len(sizes)) or real_gs(self, sizes))
    torch.manual_seed(11)
    ref = (GINet if kind == "gin" else GCN)(3, 64, 128).to(dev)
    cap = copy.deepcopy(ref)
    B = 32
    pairs = [tuple(b.to(dev) for b in p) for p in SyntheticPairBatches(B, seed=41).take(6)]
    pairs.sort(key=lambda p: p[0].x.shape[0] + p[1].x.shape[0])
    opts, reds = [], []
    for m in (ref, cap):
        opt = FusedAdam(mdist.bucketed_parameters(m), 5e-4, weight_decay=1e-5)
        mdist.broadcast_params(opt.flat)
        opts.append(opt)
        reds.append(mdist.OverlappedGradReducer(m, opt, rccl_world1))
    crit = NTXentLoss(dev, B, 0.1, True, group=rccl_world1)
    step = CapturedTrainStep(cap, opts[1], crit, node_quantum=128, edge_quantum=512, node_slack=0,
                             reducer=reds[1])
    held, big = pairs[:2], pairs[-1]
    try:
        assert step.prepare(held) >= 1 and calls == [2]
        assert step.lookup(*big) is None
        order = [held[0], big, held[1], big, held[0]]
        want = ["replay", "eager", "replay", "eager", "replay"]
        got = []
        for i, (xi, xj) in enumerate(order):
            with torch.no_grad():  # ref := cap's state
                for a, b in ((opts[0].flat, opts[1].flat), (opts[0].exp_avg, opts[1].exp_avg),
                             (opts[0].exp_avg_sq, opts[1].exp_avg_sq),
                             (opts[0]._step_dev, opts[1]._step_dev)):
                    a.copy_(b)
                for br, bc in zip(ref.batch_norms, cap.batch_norms):
                    br.running_mean.copy_(bc.running_mean)
                    br.running_var.copy_(bc.running_var)
                    br.num_batches_tracked.copy_(bc.num_batches_tracked)
            bump_param_generation()
            opts[0].zero_grad()
            reds[0].arm()
            _, z = ref.forward_pair(xi, xj)
            le = crit.forward_pair(l2_normalize(z))
            le.backward()
            reds[0].finish()
            opts[0].step()
            r0, e0, c0 = step.replays, step.eager_steps, step.captures
            lc = step(xi, xj).clone()
            torch.cuda.synchronize()
            assert step.captures == c0, "a multi-rank step must never capture on its own"
            got.append("replay" if step.replays == r0 + 1 else
                       "eager" if step.eager_steps == e0 + 1 else "?")
            assert abs(lc.item() - le.item()) <= 1e-6 * abs(le.item()), (i, got, lc.item(), le.item())
            g_rel = ((opts[1].flat_grad.double() - opts[0].flat_grad.double()).norm()
                     / opts[0].flat_grad.double().norm()).item()
            assert g_rel < 5e-5, (i, got, g_rel)
            for bc, br in zip(cap.batch_norms, ref.batch_norms):
                assert ((bc.running_var - br.running_var).norm() / br.running_var.norm()).item() < 1e-6
        assert got == want, got
        assert step.eager_steps == 2 and step.replays == 3
        # the union again (every rank's sizes): captures the big bucket, then replays it
        assert step.prepare([big]) == 1 and calls == [2, 1]
        r0 = step.replays
        step(*big)
        assert step.replays == r0 + 1
    finally:
        step.close()  # before the fixture destroys the process group
