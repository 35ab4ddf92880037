"""The captured training step (molclr_amd.graph_step) and its
device-sized kernels against the eager path.

* molclr_graph_build_dev over padded capacities equals molclr_graph_build_multi
  bit for bit on the real rows / edges; padding rows have no edges and the
  self-loop counts only.
* The device-sized segmented BatchNorm equals the host-sized one bit for bit
  on the real rows and writes zeros to the padding rows (forward and
  backward).
* A CapturedTrainStep replayed over batches of varying sizes follows the
  eager MolCLR step (zero_grad, forward_pair, F.normalize, NT-Xent, backward,
  Adam): the same loss, gradients and BatchNorm running statistics to fp32
  rounding (the split-K partition and the h3 per-tensor scales of the weight
  gradients see the padded row count), for GIN fp32 / bf16 and GCN.
"""
import copy

import pytest
import torch

from molclr_amd import _lib, ops
from molclr_amd.data import pair_graph
from molclr_amd.dataset import SyntheticPairBatches
from molclr_amd.gcn_molclr import GCN
from molclr_amd.ginet_molclr import GINet
from molclr_amd.graph_step import CapturedTrainStep, StagedPairGraph
from molclr_amd.nt_xent import NTXentLoss
from molclr_amd.ops import l2_normalize
from molclr_amd.optim import FusedAdam

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


def _to(pair, dev):
    return tuple(b.to(dev) for b in pair)


@pytest.mark.parametrize("B,pad_nodes,pad_edges", [(8, 0, 0), (64, 37, 500), (300, 1000, 4096)])
def test_graph_build_dev_matches_host(dev, B, pad_nodes, pad_edges):
    xi, xj = _to(SyntheticPairBatches(B, seed=B).next(), dev)
    ref = pair_graph(xi, xj)
    N = ref.num_nodes + pad_nodes
    E = ref.num_edges + pad_edges
    g = StagedPairGraph(dev, N, E, [B, B])
    g.stage([xi, xj])
    g.build()
    torch.cuda.synchronize()
    n, e = ref.num_nodes, ref.num_edges
    assert torch.equal(g.counts.cpu(), torch.tensor([xi.x.shape[0], xj.x.shape[0],
                                                     xi.edge_index.shape[1],
                                                     xj.edge_index.shape[1]]))
    assert torch.equal(g.x[:n].cpu(), torch.cat([xi.x, xj.x]).cpu())
    assert int(g.x[n:].abs().sum()) == 0
    assert torch.equal(g.rowptr[:n + 1], ref.rowptr)
    assert torch.equal(g.rowptr_t[:n + 1], ref.rowptr_t)
    assert bool((g.rowptr[n:] == e).all()) and bool((g.rowptr_t[n:] == e).all())
    for f in ("col", "col_t", "ecode"):
        assert torch.equal(getattr(g, f)[:e], getattr(ref, f)[:e]), f
    for f in ("nbr", "nbr_t"):
        assert torch.equal(getattr(g, f)[:4 * n], getattr(ref, f)[:4 * n]), f
        assert int(getattr(g, f)[4 * n:].abs().sum()) == 0, f
    assert torch.equal(g.ecount[:8 * n], ref.ecount)
    pad = g.ecount[8 * n:].view(-1, 8).cpu()
    assert torch.equal(pad, torch.tensor([0, 0, 0, 0, 1, 1, 0, 0]).expand_as(pad).int())
    assert torch.equal(g.graph_ptr, ref.graph_ptr)
    assert int(g.status.item()) == 0 and int(ref.status.item()) == 0


def test_stage_rejects_overflow(dev):
    xi, xj = _to(SyntheticPairBatches(16, seed=3).next(), dev)
    n = xi.x.shape[0] + xj.x.shape[0]
    e = xi.edge_index.shape[1] + xj.edge_index.shape[1]
    with pytest.raises(_lib.MolclrError):
        StagedPairGraph(dev, n - 1, e, [16, 16]).stage([xi, xj])
    with pytest.raises(_lib.MolclrError):
        StagedPairGraph(dev, n, e - 1, [16, 16]).stage([xi, xj])


@pytest.mark.parametrize("dtype", [_lib.DTYPE_F32, _lib.DTYPE_BF16])
@pytest.mark.parametrize("rows,pad,D", [((700, 900), 300, 64), ((15000, 15300), 1200, 300),
                                        # c5-sized: > 512 partitions per segment (band 2 at
                                        # D = 512: 32 rows per partition), 1730 in all
                                        ((27700, 27650), 600, 512)])
def test_batchnorm_dev_matches_host(dev, dtype, rows, pad, D):
    lib = _lib.load()
    st = ops._stream(torch.empty(1, device=dev))
    n = sum(rows)
    cap = n + pad
    g = torch.Generator().manual_seed(D + pad)
    z32 = torch.randn(cap, D, generator=g).to(dev) * 3 + 1
    dy32 = torch.randn(cap, D, generator=g).to(dev)
    tdt = torch.bfloat16 if dtype == _lib.DTYPE_BF16 else torch.float32
    z, dy = z32.to(tdt).contiguous(), dy32.to(tdt).contiguous()
    gamma = torch.rand(D, generator=g).to(dev) + 0.5
    beta = torch.randn(D, generator=g).to(dev)
    seg = (ctypes_i64 := __import__("ctypes").c_int64 * 2)(*rows)
    drows = torch.tensor(rows, dtype=torch.long, device=dev)
    out = {}
    for mode in ("host", "dev"):
        rm, rv = torch.zeros(D, device=dev), torch.ones(D, device=dev)
        nbt = torch.zeros(1, dtype=torch.long, device=dev)
        y = torch.full_like(z, 7.0)
        mean, inv = torch.empty(2, D, device=dev), torch.empty(2, D, device=dev)
        dz = torch.full_like(z, 7.0)
        dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        if mode == "host":
            wsb = lib.molclr_batchnorm_seg_workspace_bytes(2, seg, D)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            assert lib.molclr_batchnorm_seg_fwd(
                z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                nbt.data_ptr(), y.data_ptr(), mean.data_ptr(), inv.data_ptr(), 2, seg, D, dtype,
                0.1, 1e-5, 1, 1, ws.data_ptr(), wsb, st) == 0
            assert lib.molclr_batchnorm_seg_bwd(
                dy.data_ptr(), z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
                inv.data_ptr(), dz.data_ptr(), dg.data_ptr(), db.data_ptr(), 2, seg, D, dtype, 1,
                0, ws.data_ptr(), wsb, st) == 0
        else:
            wsb = lib.molclr_batchnorm_seg_dev_workspace_bytes(2, cap, D)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            assert lib.molclr_batchnorm_seg_fwd_dev(
                z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                nbt.data_ptr(), y.data_ptr(), mean.data_ptr(), inv.data_ptr(), 2,
                drows.data_ptr(), cap, D, dtype, 0.1, 1e-5, 1, 1, ws.data_ptr(), wsb, st) == 0
            assert lib.molclr_batchnorm_seg_bwd_dev(
                dy.data_ptr(), z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
                inv.data_ptr(), dz.data_ptr(), dg.data_ptr(), db.data_ptr(), 2, drows.data_ptr(),
                cap, D, dtype, 1, 0, None, None, ws.data_ptr(), wsb, st) == 0
        torch.cuda.synchronize()
        out[mode] = dict(y=y, dz=dz, rm=rm, rv=rv, nbt=nbt, mean=mean, inv=inv, dg=dg, db=db)
    h, d = out["host"], out["dev"]
    for k in ("rm", "rv", "nbt", "mean", "inv", "dg", "db"):
        assert torch.equal(h[k], d[k]), k
    assert torch.equal(h["y"][:n], d["y"][:n]) and torch.equal(h["dz"][:n], d["dz"][:n])
    assert int(d["y"][n:].float().abs().sum()) == 0 and int(d["dz"][n:].float().abs().sum()) == 0


def _make(kind, seed):
    torch.manual_seed(seed)
    if kind == "gcn":
        return GCN(num_layer=3, emb_dim=64, feat_dim=64)
    return GINet(num_layer=3, emb_dim=64, feat_dim=64, precision="bf16" if kind == "bf16" else "fp32")


def _eager_step(model, opt, crit, xi, xj):
    opt.zero_grad()
    _, z = model.forward_pair(xi, xj)
    loss = crit.forward_pair(l2_normalize(z))
    loss.backward()
    opt.step()
    return loss.detach().clone()


def _sync(ref, opt_r, cap, opt_c):
    """ref's optimizer and BatchNorm state := cap's (Adam turns rounding-level
    gradient differences into +-lr steps, so trajectories are compared one
    step at a time from the same state)."""
    with torch.no_grad():
        for a, b in ((opt_r.flat, opt_c.flat), (opt_r.exp_avg, opt_c.exp_avg),
                     (opt_r.exp_avg_sq, opt_c.exp_avg_sq), (opt_r._step_dev, opt_c._step_dev)):
            a.copy_(b)
        for br, bc in zip(ref.batch_norms, cap.batch_norms):
            br.running_mean.copy_(bc.running_mean)
            br.running_var.copy_(bc.running_var)
            br.num_batches_tracked.copy_(bc.num_batches_tracked)
    ops.bump_param_generation()


@pytest.mark.parametrize("kind", ["gin", "bf16", "gcn"])
def test_captured_step_follows_eager(dev, kind):
    """Every replay (first captures of several buckets and later replays of
    them) against an eager step from the same state: the forward is the same
    on the real rows (loss to 1e-6), the gradients differ only by the weight
    gradients' summation order over the padded rows (norm-wise 1e-5; bf16
    1e-4), the running statistics by nothing but that."""
    B = 32
    batches = [_to(p, dev) for p in SyntheticPairBatches(B, seed=11).take(6)]
    ref = _make(kind, 5).to(dev)
    cap = copy.deepcopy(ref)
    opt_r = FusedAdam(ref.parameters(), 5e-4, weight_decay=1e-5)
    opt_c = FusedAdam(cap.parameters(), 5e-4, weight_decay=1e-5)
    crit = NTXentLoss(dev, B, 0.1, True)
    # small quanta: several buckets, several captures, replays of each
    step = CapturedTrainStep(cap, opt_c, crit, node_quantum=128, edge_quantum=512, node_slack=0)
    tol_grad = 1e-5 if kind != "bf16" else 1e-4
    for i, (xi, xj) in enumerate(batches + batches[:3]):
        _sync(ref, opt_r, cap, opt_c)
        lr_ = _eager_step(ref, opt_r, crit, xi, xj)
        lc = step(xi, xj).clone()
        torch.cuda.synchronize()
        assert abs(lc.item() - lr_.item()) <= 1e-6 * abs(lr_.item()), (i, lc.item(), lr_.item())
        r = rel(opt_c.flat_grad, opt_r.flat_grad)
        if r >= tol_grad:
            per = sorted(((rel(pc.grad, pr.grad), n, pc.grad.norm().item(), pr.grad.norm().item())
                          for (n, pc), pr in zip(cap.named_parameters(), ref.parameters())),
                         reverse=True)[:8]
            raise AssertionError(f"step {i}: rel {r:.3g}, captures {step.captures}, replays "
                                 f"{step.replays}; worst (rel, name, |cap|, |eager|): {per}")
        for bc, br in zip(cap.batch_norms, ref.batch_norms):
            assert rel(bc.running_mean, br.running_mean) < 1e-6, i
            assert rel(bc.running_var, br.running_var) < 1e-6, i
            assert int(bc.num_batches_tracked) == int(br.num_batches_tracked), i
        assert opt_c.steps_taken == opt_r.steps_taken
    assert step.captures >= 2
    # eager use after replays sees the replayed weights (planes refreshed)
    _sync(ref, opt_r, cap, opt_c)
    cap.eval()
    ref.eval()
    with torch.no_grad():
        xi, xj = batches[0]
        assert torch.equal(cap(xi)[1], ref(xi)[1])
    # the captured graph's status word is the batch's
    step.last_graph.check()


def test_captured_step_lr_follows_scheduler(dev):
    B = 16
    batches = [_to(p, dev) for p in SyntheticPairBatches(B, seed=2).take(3)]
    model = _make("gin", 1).to(dev)
    opt = FusedAdam(model.parameters(), 1e-3)
    step = CapturedTrainStep(model, opt, NTXentLoss(dev, B, 0.1, True))
    xi, xj = batches[0]
    step(xi, xj)
    before = opt.flat.clone()
    opt.param_groups[0]["lr"] = 0.0  # a replay must read the new learning rate
    step(xi, xj)
    torch.cuda.synchronize()
    assert torch.equal(opt.flat, before)
    assert opt.steps_taken == 2


def test_capacity_fit_lookup_and_prepare(dev):
    """A pair replays on the smallest captured graph that holds it within the
    node slack; prepare() captures ahead of time, so the steps after it
    capture nothing; a replay on a larger graph (padding rows) still follows
    the eager step."""
    B = 32
    pairs = [_to(p, dev) for p in SyntheticPairBatches(B, seed=21).take(8)]
    ref = _make("gin", 3).to(dev)
    cap = copy.deepcopy(ref)
    opt_r = FusedAdam(ref.parameters(), 5e-4, weight_decay=1e-5)
    opt_c = FusedAdam(cap.parameters(), 5e-4, weight_decay=1e-5)
    crit = NTXentLoss(dev, B, 0.1, True)
    # a slack of ~a quarter of the pairs' rows (B = 32: ~1.9k nodes per pair);
    # the largest pair's graph serves every smaller one within it
    step = CapturedTrainStep(cap, opt_c, crit, node_quantum=64, edge_quantum=256,
                             node_slack=512)
    order = sorted(pairs, key=lambda p: -(p[0].x.shape[0] + p[1].x.shape[0]))
    assert step.prepare(order[:1]) == 1
    biggest = step.lookup(*order[0])
    for p in order:
        ent = step.lookup(*p)
        if ent is not None:
            assert ent is biggest
    n_before = step.captures
    step.prepare(pairs)
    n_prepared = step.captures
    for xi, xj in pairs + pairs[:2]:
        _sync(ref, opt_r, cap, opt_c)
        lr_ = _eager_step(ref, opt_r, crit, xi, xj)
        lc = step(xi, xj).clone()
        torch.cuda.synchronize()
        assert abs(lc.item() - lr_.item()) <= 1e-6 * abs(lr_.item())
        # per parameter; the pre-BatchNorm biases have an exact gradient of 0
        # and hold rounding noise only (tests/test_gpu_models.py: pre_bn_bias).
        # Bound: the padded rows change the weight gradients' split-K partition
        # (w6_plan derives it from the row count), i.e. the fp32 summation
        # order of dW = dY^T X over ~2k rows with cancellation: measured up to
        # 2.8e-5 here, against ~1e-3 for the reference's own fp32 vs fp64
        # (paired vs two-call gradients)
        bad = []
        for (name, pc), pr in zip(cap.named_parameters(), ref.parameters()):
            if name.endswith("mlp.2.bias"):
                continue
            r = rel(pc.grad, pr.grad)
            if r > 5e-5:
                bad.append((name, r, pc.grad.norm().item(), pr.grad.norm().item()))
        assert not bad, bad
    assert step.captures == n_prepared  # nothing captured after prepare()
    assert step.replays == len(pairs) + 2
    # a tight slack refuses the oversized graph and captures an exact one
    tight = CapturedTrainStep(cap, opt_c, crit, node_quantum=64, edge_quantum=256, node_slack=0)
    tight.prepare(order[:1])
    small = order[-1]
    assert tight.lookup(*small) is None
    tight.prepare([small])
    assert tight.captures == 2 and tight.lookup(*small) is not None


class _Poison:
    """Every floating-point torch.empty / empty_like of the library's Python
    code (executor arenas, GEMM / BatchNorm outputs, NT-Xent buffers, graph
    capacities) comes back filled with ``value`` -- inside a capture too, as a
    fill node that runs on every replay.  A kernel that reads memory it was
    never given a value for then sees 0, a huge finite number or NaN
    depending on the poison, and the step's results change with it."""

    def __init__(self, value):
        self.value = value

    def __enter__(self):
        self._empty, self._like = torch.empty, torch.empty_like
        value, real_empty, real_like = self.value, self._empty, self._like

        def empty(*a, **k):
            t = real_empty(*a, **k)
            if t.is_cuda and t.is_floating_point():
                t.fill_(value)
            return t

        def empty_like(x, *a, **k):
            t = real_like(x, *a, **k)
            if t.is_cuda and t.is_floating_point():
                t.fill_(value)
            return t
        torch.empty, torch.empty_like = empty, empty_like
        return self

    def __exit__(self, *exc):
        torch.empty, torch.empty_like = self._empty, self._like


def _poisoned_run(dev, kind, value, batches, captured):
    with _Poison(value):
        model = _make(kind, 9).to(dev)
        opt = FusedAdam(model.parameters(), 5e-4, weight_decay=1e-5)
        crit = NTXentLoss(dev, 32, 0.1, True)
        losses = []
        if captured:
            step = CapturedTrainStep(model, opt, crit, node_quantum=128, edge_quantum=512,
                                     node_slack=0)
            for xi, xj in batches:
                losses.append(step(xi, xj).clone())
            grads = opt.flat_grad.clone()
            step.close()
        else:
            for xi, xj in batches:
                losses.append(_eager_step(model, opt, crit, xi, xj))
            grads = opt.flat_grad.clone()
        torch.cuda.synchronize()
        bn = [(b.running_mean.clone(), b.running_var.clone()) for b in model.batch_norms]
        return torch.stack(losses), grads, opt.flat.clone(), bn


@pytest.mark.parametrize("captured", [False, True], ids=["eager", "captured"])
@pytest.mark.parametrize("kind", ["gin", "bf16", "gcn"])
def test_no_uninitialised_reads(dev, kind, captured):
    """The step's results do not depend on what its buffers held before:
    with every fresh floating-point buffer pre-filled with 0, 3e38 or NaN,
    the losses, the last step's gradients, the parameters after Adam and the
    BatchNorm running statistics are bit-identical.  Captured: several
    capacity buckets, replays of smaller batches on a graph whose padding rows
    then lie between the batch and the capacity (the captured data-parallel
    step once lost its MLP weight gradients after other tests had run in the
    same process: a read of stale memory is the class of fault that depends on
    process history)."""
    batches = [_to(p, dev) for p in SyntheticPairBatches(32, seed=41).take(4)]
    order = batches + [batches[0], batches[2], batches[1]]
    runs = {v: _poisoned_run(dev, kind, v, order, captured) for v in (0.0, 3e38, float("nan"))}
    base = runs[0.0]
    for v, r in runs.items():
        assert torch.equal(r[0], base[0]), (v, r[0], base[0])
        assert torch.equal(r[1], base[1]), (v, rel(r[1], base[1]))
        assert torch.equal(r[2], base[2]), v
        for (m, s), (m0, s0) in zip(r[3], base[3]):
            assert torch.equal(m, m0) and torch.equal(s, s0), v


@pytest.mark.parametrize("captured", [False, True], ids=["eager", "captured"])
@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_side_stream_head_gradients_bit_identical(dev, kind, captured, monkeypatch):
    """The readout heads' weight gradients run on a side stream
    (ops.linear_bwd side=True, joined by the encoder backward and Adam): the
    same kernels in the same per-stream order, so losses, gradients, parameters
    and running statistics equal the one-stream step's bit for bit, eager and
    as a captured graph (fork / join inside the capture)."""
    from molclr_amd import ops
    batches = [_to(p, dev) for p in SyntheticPairBatches(32, seed=43).take(3)]
    order = batches + [batches[0]]
    monkeypatch.setattr(ops, "SIDE_WGRAD", False)
    one = _poisoned_run(dev, kind, 0.0, order, captured)
    monkeypatch.setattr(ops, "SIDE_WGRAD", True)
    two = _poisoned_run(dev, kind, 0.0, order, captured)
    assert not ops._SIDE_PENDING
    assert torch.equal(one[0], two[0]), (one[0], two[0])
    assert torch.equal(one[1], two[1]), rel(one[1], two[1])
    assert torch.equal(one[2], two[2])
    for (m, s), (m0, s0) in zip(one[3], two[3]):
        assert torch.equal(m, m0) and torch.equal(s, s0)


def test_captured_zeroing_takes_effect(dev):
    """The library zeroes buffers (h3 max slots, pooled-gradient rows, edge
    histograms) with kernels (common.h zero_async), not hipMemsetAsync: a
    memset node that follows a kernel node in a captured graph did not take
    effect on replays on this runtime (profiles/r5_capture_memset_probe.txt:
    299 of 300 replays), which left the h3 max slots stale -- the round-4
    captured data-parallel failure.  Region poisoned before each replay; the
    zeroing and a kernel reading the zeroed region after it must see 0."""
    lib = _lib.load()
    x = torch.randn(16, device=dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        slot = torch.empty(ops.MAX_SLOT, device=dev)
        y = x * 2  # a kernel node first: the memset node then follows it
        # rows = 0: the call only zeroes its max slot
        assert lib.molclr_absmax_f32(y.data_ptr(), 0, 0, 1, slot.data_ptr(), 0,
                                     ops._stream(y)) == 0
        copy = slot * 1.0
    for _ in range(20):
        slot.fill_(3e38)
        copy.fill_(3e38)
        g.replay()
        torch.cuda.synchronize()
        assert int((slot != 0).sum()) == 0 and int((copy != 0).sum()) == 0
