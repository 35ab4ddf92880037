"""Data-parallel logic on CPU with gloo, world size 2.

* The row-sharded NT-Xent the kernels implement — each rank owns its
  [zj_local; zi_local] rows, all-gathers the projections into the reference's
  global order [zj_all; zi_all] and the per-row lse, and computes the exact
  gradient of its own rows (symmetric W, no column-gradient exchange) —
  reproduces the single-process reference NTXentLoss on the concatenated
  batch, loss and gradients.
* The product's exchange helpers (molclr_amd.distributed.gather_rows /
  gather_lse / global_row_index, what ops._NTXent calls) produce the
  reference's global order.
* molclr_amd.distributed: init() from the torchrun environment, the flat
  gradient SUM all-reduce and the parameter broadcast.
* Data parallel input: MoleculeDatasetWrapper gives each rank a disjoint,
  equally sized shard, reshuffled every epoch (identical per-rank
  data made every row meet copies of itself as negatives).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ntxent_math
from oracle.reference_cpu import RefNTXentLoss

WORLD = 2
B_LOCAL, C, T = 16, 64, 0.1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs():
    rng = np.random.default_rng(0)
    zi = rng.standard_normal((WORLD * B_LOCAL, C)).astype(np.float32)
    zj = (0.5 * zi + rng.standard_normal((WORLD * B_LOCAL, C))).astype(np.float32)
    return zi, zj


def _worker(rank, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    from molclr_amd import distributed as mdist
    r, w, dev = mdist.init(backend="gloo")
    assert (r, w, dev.type) == (rank, WORLD, "cpu")
    zi, zj = _inputs()
    sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
    B = WORLD * B_LOCAL
    # local rows [zj_local; zi_local], global indices
    R_local = np.concatenate([zj[sl], zi[sl]], 0)
    rh, nrm = ntxent_math.prep(R_local, True)
    # the product's exchange (molclr_amd.distributed, as ops._NTXent calls it):
    # one gather of [zj_local; zi_local] into [zj_all; zi_all], global row ids
    gidx = mdist.global_row_index(B_LOCAL, rank, WORLD, "cpu").numpy().astype(np.int64)
    assert np.array_equal(gidx, np.concatenate([np.arange(B_LOCAL) + rank * B_LOCAL,
                                                np.arange(B_LOCAL) + rank * B_LOCAL + B]))
    cols = mdist.gather_rows(torch.from_numpy(rh)).numpy()
    Rall = np.concatenate([zj, zi], 0)
    assert np.allclose(cols, ntxent_math.prep(Rall, True)[0])
    lse, loss_rows = ntxent_math.rows_forward(rh, gidx, cols, B, T)
    lse_cols = mdist.gather_lse(torch.from_numpy(lse)).numpy()
    assert np.allclose(lse_cols, ntxent_math.rows_forward(cols, np.arange(2 * B), cols, B, T)[0])
    loss = torch.tensor([loss_rows.sum()])
    dist.all_reduce(loss)
    # ops._NTXent's form: lse gather and the loss SUM in one all-gather
    lse2, loss2 = mdist.gather_lse_and_sum(torch.from_numpy(lse),
                                           torch.tensor(loss_rows.sum(), dtype=torch.float32))
    assert np.array_equal(lse2.numpy(), lse_cols)
    assert np.isclose(loss2.item(), loss.item(), rtol=1e-6)
    drh = ntxent_math.rows_backward(rh, gidx, cols, lse_cols, B, T)
    dR = ntxent_math.prep_bwd(drh, rh, nrm, True)
    # data sharding: disjoint, equally sized per-rank shards every epoch
    from molclr_amd.dataset import MoleculeDatasetWrapper
    w = MoleculeDatasetWrapper(8, 0, 0.2, "synthetic:120", seed=3, views="host")
    tr, va = w.get_data_loaders()
    ids = []
    for epoch in range(2):
        ids.append(list(tr.sampler))
    first = next(iter(tr))[0]
    nb = torch.tensor([len(tr), len(va)])
    nbs = [torch.zeros(2, dtype=torch.long) for _ in range(WORLD)]
    dist.all_gather(nbs, nb)
    shard = torch.tensor(sorted(ids[0]))
    shards = [torch.zeros_like(shard) for _ in range(WORLD)]
    dist.all_gather(shards, shard)
    xs = torch.tensor([first.x.shape[0]])
    sizes = [torch.zeros_like(xs) for _ in range(WORLD)]
    dist.all_gather(sizes, xs)
    sharding = ([n.tolist() for n in nbs], [s.tolist() for s in shards], ids[0] != ids[1])
    # gradient reduction + broadcast helpers on flat buffers
    flat = torch.full((10,), float(rank + 1))
    mdist.allreduce_grads(flat)
    p = torch.full((4,), float(rank))
    mdist.broadcast_params(p)
    out_q.put((rank, float(loss.item()), dR[B_LOCAL:], dR[:B_LOCAL], flat.tolist(), p.tolist(),
               sharding))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_ntxent_matches_single_process_reference():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(WORLD)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    zi, zj = _inputs()
    a = torch.from_numpy(zi).requires_grad_(True)
    b = torch.from_numpy(zj).requires_grad_(True)
    ref = RefNTXentLoss("cpu", WORLD * B_LOCAL, T, True)(a, b)
    ref.backward()
    dzi = np.concatenate([r[2] for r in res], 0)
    dzj = np.concatenate([r[3] for r in res], 0)
    for r in res:
        assert abs(r[1] - ref.item()) < 1e-5 * ref.item()
        assert r[4] == [3.0] * 10        # SUM over ranks 1 + 2
        assert r[5] == [0.0] * 4         # rank 0's values broadcast
    nbs, shards, reshuffled = res[0][6]
    assert nbs[0] == nbs[1] and nbs[0][0] > 0       # equal batch counts per rank
    assert not set(shards[0]) & set(shards[1])      # disjoint molecule shards
    assert reshuffled                                 # a new permutation every epoch
    assert np.linalg.norm(dzi - a.grad.numpy()) <= 1e-5 * np.linalg.norm(a.grad.numpy())
    assert np.linalg.norm(dzj - b.grad.numpy()) <= 1e-5 * np.linalg.norm(b.grad.numpy())


class _FlatLayout:
    """FusedAdam's flat-buffer layout (4-aligned slots in parameter order)
    without its GPU-only state: what OverlappedGradReducer reads."""

    def __init__(self, params):
        self.views, off = [], 0
        for p in params:
            self.views.append((p, off, p.numel()))
            off += (p.numel() + 3) // 4 * 4
        self.flat_grad = torch.zeros(off)


def _reducer_worker(rank, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    from molclr_amd import distributed as mdist
    from molclr_amd import ops
    from molclr_amd.ginet_molclr import GINet
    mdist.init(backend="gloo")
    torch.manual_seed(0)
    model = GINet(3, 16, 32)
    names = {id(p): n for n, p in model.named_parameters()}
    order = [[names[id(p)] for p in b] for b in mdist.gradient_buckets(model)]
    layout = _FlatLayout(mdist.bucketed_parameters(model))
    red = mdist.OverlappedGradReducer(model, layout, dist.group.WORLD)
    n = layout.flat_grad.numel()
    base = torch.arange(n, dtype=torch.float32)
    # the protocol the encoder backward drives (ops._grad_events)
    layout.flat_grad.copy_(base * (rank + 1))
    red.arm()
    assert ops._GRAD_HOOK is red
    red.encoder_backward_begin()
    try:
        red.encoder_backward_begin()  # a second encoder backward in one step
        second = "accepted"
    except RuntimeError:
        second = "refused"
    red.encoder_backward_enqueued()
    red.finish()
    bucketed = layout.flat_grad.clone()
    # no executor backward in the step: one collective over the whole buffer
    layout.flat_grad.copy_(base * (rank + 1))
    red.arm()
    red.finish()
    assert ops._GRAD_HOOK is None
    out_q.put((rank, order, red.slices, n, bucketed.tolist(), layout.flat_grad.tolist(), second))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_overlapped_grad_reducer_buckets_and_sums():
    """molclr_amd.distributed.OverlappedGradReducer under gloo, world 2: the
    buckets follow the backward's completion order (heads, layer L-1 .. 0,
    atom embeddings), tile the flat gradient buffer exactly as contiguous
    disjoint slices, and the bucketed reduction equals one SUM all-reduce."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_reducer_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(WORLD)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, order, slices, n, bucketed, whole, second = res[0]
    assert all(x.startswith(("feat_lin.", "out_lin.")) for x in order[0])
    for k, l in enumerate((2, 1, 0)):
        assert order[1 + k] and all(x.startswith((f"gnns.{l}.", f"batch_norms.{l}."))
                                    for x in order[1 + k])
    assert sorted(order[-1]) == ["x_embedding1.weight", "x_embedding2.weight"]
    assert slices[0][0] == 0 and slices[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(slices, slices[1:]))  # contiguous, disjoint
    expect = [3.0 * i for i in range(n)]  # SUM of ranks' (rank + 1) * arange
    for r in res:
        assert r[4] == expect and r[5] == expect
        assert r[6] == "refused"


def _global_sizes_worker(rank, world, port, q):
    import types

    import torch.distributed as dist

    from molclr_amd.graph_step import CapturedTrainStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fake = types.SimpleNamespace(group=dist.group.WORLD, device=torch.device("cpu"))
        local = [[(3000, 9000), (2800, 8000)], [(3100, 9100)], []][rank]
        q.put((rank, CapturedTrainStep._global_sizes(fake, local)))
    finally:
        dist.destroy_process_group()


def test_capture_sizes_union_across_ranks():
    """Data-parallel captures happen in lockstep: every rank gets the union of
    all ranks' (nodes, edges) sizes, largest first, whatever its own list
    (graph_step.CapturedTrainStep._global_sizes over gloo, world 3, one rank
    with no sizes)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_global_sizes_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    want = [(3100, 9100), (3000, 9000), (2800, 8000)]
    assert all(got[r] == want for r in range(3)), got


def _plan_worker(rank, world, port, q):
    """CapturedTrainStep's capture planning (lookup / prepare_sizes / replay /
    eviction) on a stub whose captures record nothing (no GPU): what each
    rank decides, step by step."""
    import types
    from collections import OrderedDict

    import torch.distributed as dist

    from molclr_amd.graph_step import CapturedTrainStep, _Captured
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = object.__new__(CapturedTrainStep)
        st.group = dist.group.WORLD
        st.device = torch.device("cpu")
        st.node_quantum, st.edge_quantum, st.node_slack, st.edge_headroom = 256, 2048, 512, 0.04
        st.max_graphs = 2
        st._graphs = OrderedDict()
        st.captures = st.replays = st.eager_steps = 0
        st.loss, st.last_graph = torch.zeros(()), None
        st.optimizer = types.SimpleNamespace(sync_lr=lambda: None)
        log = []

        def capture(key, pair=None):
            st.captures += 1
            log.append(("capture", key[:2]))
            g = types.SimpleNamespace(num_nodes=key[0], num_edges=key[1],
                                      graphs_per_segment=list(key[2:]), stage=lambda v: None)
            return _Captured(g, types.SimpleNamespace(replay=lambda: None))

        def eager(xis, xjs):
            st.eager_steps += 1
            log.append(("eager",))
            return None

        st._capture, st._eager = capture, eager

        class _View:
            def __init__(self, n, e):
                self.x = torch.empty(n, 0)
                self.edge_index = torch.empty(2, e)
                self.num_graphs = 4

        # three size classes 1024 nodes apart (each needs its own capture)
        sizes = [(1000, 3000), (2000, 6000), (3000, 9000)]
        st.prepare_sizes(sizes[:2], 4, 4)            # captures 2000, then 1000
        # ranks replay DIFFERENT buckets (rank 0 the large one, rank 1 the small)
        mine = sizes[1] if rank == 0 else sizes[0]
        for _ in range(3):
            st(_View(*mine), _View(0, 0))
        st.prepare_sizes([sizes[2]], 4, 4)           # a third capture: one eviction
        after = [(g.graph.num_nodes, g.graph.num_edges) for g in st._graphs.values()]
        # a batch of every class on every rank: replay or (lockstep-safe) eager
        for n, e in sizes:
            st(_View(n, e), _View(0, 0))
        st.prepare_sizes(sizes, 4, 4)                # the union again
        final = [(g.graph.num_nodes, g.graph.num_edges) for g in st._graphs.values()]
        q.put((rank, after, final, st.captures, log))
    finally:
        dist.destroy_process_group()


def test_capture_plan_stays_in_lockstep_when_ranks_replay_different_buckets():
    """replays used to reorder the LRU, so after an eviction ranks
    could hold different graph sets and one rank would capture (recording
    collectives) while another did not.  With several ranks, eviction now
    follows capture order: every rank keeps the same graphs and makes the
    same capture decisions, whatever buckets it replayed (gloo, world 2,
    max_graphs 2)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a0, f0, c0, log0 = got[0]
    a1, f1, c1, log1 = got[1]
    assert a0 == a1 and f0 == f1 and c0 == c1
    caps = lambda log: [e for e in log if e[0] == "capture"]  # noqa: E731
    assert caps(log0) == caps(log1)
    assert len(a0) == 2  # max_graphs
