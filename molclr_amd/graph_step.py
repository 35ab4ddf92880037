"""The pre-training step captured as HIP graphs.

The reference's hot loop (molclr.py:107-128) enqueues, per step: the graph of
both views, the encoder forward, F.normalize, NT-Xent, the backward and the
Adam update.  Here that is ~150 kernel launches (the encoder executors issue
most of them from C++), ~1.5 ms of host time per step.  This module captures
the whole step ONCE per batch-size bucket as a HIP graph (torch.cuda.CUDAGraph
over the library's launches) and replays it: the host cost per step becomes
one staging launch plus one graph launch.

Batches vary in size, a graph does not.  The step therefore runs over
fixed-capacity buffers:

* ``StagedPairGraph`` holds staging buffers for both views' PyG fields and the
  graph outputs, sized by a bucket's capacities (nodes rounded up to
  ``node_quantum``, edges to ``edge_quantum``).  Before a replay,
  ``molclr_stage_segments`` copies the batch in (one launch) and writes the
  views' real node / edge counts to the device; inside the graph
  ``molclr_graph_build_dev`` and the BatchNorm kernels read those counts.
* Rows past the real nodes are padding: atoms (0, 0) without edges, outside
  every graph, zero BatchNorm output and zero gradient, so they change no
  parameter gradient, statistic or loss (tests/test_gpu_graph_step.py holds
  the replayed step to the eager one).
* The learning rate and Adam's step counter already live on the device
  (FusedAdam); the weight planes are regenerated inside the graph.

Data parallel (one process per GPU, RCCL): the step's collectives are
captured with it -- NT-Xent's two all-gathers, and the bucketed gradient
all-reduces of OverlappedGradReducer, which wait on the encoder backward's
per-layer events from a side stream and are joined before Adam, exactly as
in the eager step (RCCL kernels are captured into the HIP graph like any
other launch).  Every step issues the same collectives in the same order
whatever graph a rank replays (the bucket sizes and the gathered NT-Xent
shapes do not depend on the batch's atom count), so ranks may replay
different buckets.  Captures themselves happen in lockstep: prepare /
prepare_sizes capture the union of every rank's sizes on every rank, and a
rank whose batch no captured graph holds steps eagerly (same collectives)
instead of capturing alone.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import torch

from . import _lib, ops
from .data import DeviceGraph, _num_graphs_of


def _round_up(n: int, q: int) -> int:
    return max(q, (int(n) + q - 1) // q * q)


class StagedPairGraph(DeviceGraph):
    """A DeviceGraph over fixed capacities (node_cap rows, edge_cap edge slots)
    whose views are staged in before every use (``stage``) and whose build
    (``build``) reads the real sizes on the device -- both capturable."""

    def __init__(self, device, node_cap: int, edge_cap: int, graphs_per_segment):
        self.device = device
        self.nseg = len(graphs_per_segment)
        i64 = dict(dtype=torch.long, device=device)
        i32 = dict(dtype=torch.int32, device=device)
        N, E, G = int(node_cap), int(edge_cap), int(sum(graphs_per_segment))
        self.num_nodes, self.num_edges, self.num_graphs = N, E, G
        self.graphs_per_segment = [int(g) for g in graphs_per_segment]
        self.segment_nodes = None  # on the device: self.counts[:nseg]
        # staging: every segment gets the full capacity (a few MB)
        self.st_ei = [torch.zeros(2, E, **i64) for _ in range(self.nseg)]
        self.st_ea = [torch.zeros(E, 2, **i64) for _ in range(self.nseg)]
        self.st_batch = [torch.zeros(N, **i64) for _ in range(self.nseg)]
        self.x = torch.zeros(N, 2, **i64)
        self.counts = torch.zeros(2 * self.nseg, **i64)
        self._dst = (_lib.StagedSegmentC * self.nseg)()
        for q in range(self.nseg):
            self._dst[q] = _lib.StagedSegmentC(self.st_ei[q].data_ptr(), self.st_ea[q].data_ptr(),
                                               self.st_batch[q].data_ptr(), N, E,
                                               self.graphs_per_segment[q])
        self.rowptr = torch.empty(N + 1, **i32)
        self.col = torch.empty(E, **i32)
        self.ecode = torch.empty(E, dtype=torch.uint8, device=device)
        self.rowptr_t = torch.empty(N + 1, **i32)
        self.col_t = torch.empty(E, **i32)
        self.nbr = torch.empty(N * 4, **i32)
        self.nbr_t = torch.empty(N * 4, **i32)
        self.ecount = torch.empty(N * 8, **i32)
        self.graph_ptr = torch.empty(G + 1, **i32)
        self.status = torch.zeros(1, **i32)
        self._ws_bytes = _lib.query("molclr_graph_build_workspace_bytes", N, E)
        self._ws = torch.empty(self._ws_bytes, dtype=torch.uint8, device=device)
        self._keep = []

    def fits(self, views) -> bool:
        n = sum(int(v.x.shape[0]) for v in views)
        e = sum(int(v.edge_index.shape[1]) for v in views)
        return (n <= self.num_nodes and e <= self.num_edges
                and [_num_graphs_of(v) for v in views] == self.graphs_per_segment)

    def stage(self, views) -> None:
        """Copy the views' x / edge_index / edge_attr / batch in (one launch on
        the current stream); the inputs must stay alive until it has run."""
        if len(views) != self.nseg:
            raise ValueError(f"StagedPairGraph: {len(views)} views, built for {self.nseg}")
        src = (_lib.StageSourceC * self.nseg)()
        keep = []
        for q, d in enumerate(views):
            if _num_graphs_of(d) != self.graphs_per_segment[q]:
                raise ValueError("StagedPairGraph: a view's graph count changed "
                                 f"({_num_graphs_of(d)} vs {self.graphs_per_segment[q]})")
            x = d.x.to(torch.long).contiguous()
            ei = d.edge_index.to(torch.long).contiguous()
            ea = d.edge_attr.to(torch.long).contiguous()
            b = getattr(d, "batch", None)
            if b is None:
                b = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
            b = b.to(torch.long).contiguous()
            keep += [x, ei, ea, b]
            src[q] = _lib.StageSourceC(x.data_ptr(), ei.data_ptr(), ea.data_ptr(), b.data_ptr(),
                                       int(x.shape[0]), int(ei.shape[1]))
        _lib.call("molclr_stage_segments", self.nseg, ctypes.addressof(src),
                  ctypes.addressof(self._dst), self.x.data_ptr(), self.num_nodes, self.num_edges,
                  self.counts.data_ptr(), _lib.stream_of(self.device))
        self._keep = keep  # until the next stage: the copy is asynchronous

    def build(self) -> None:
        """molclr_graph_build_dev on the current stream (capturable)."""
        _lib.call("molclr_graph_build_dev", self.nseg, ctypes.addressof(self._dst),
                  self.counts.data_ptr(), self.num_nodes, self.num_edges,
                  self.rowptr.data_ptr(), self.col.data_ptr(), self.ecode.data_ptr(),
                  self.rowptr_t.data_ptr(), self.col_t.data_ptr(), self.nbr.data_ptr(),
                  self.nbr_t.data_ptr(), self.ecount.data_ptr(), self.graph_ptr.data_ptr(),
                  self.status.data_ptr(), self._ws.data_ptr(), self._ws_bytes,
                  _lib.stream_of(self.device))

    def cstruct(self):
        c = getattr(self, "_cstruct", None)
        if c is None:
            c = _lib.DeviceGraphC(self.num_nodes, self.num_edges, self.num_graphs, *[
                t.data_ptr() for t in (self.rowptr, self.col, self.rowptr_t, self.col_t,
                                       self.ecount, self.graph_ptr, self.ecode, self.nbr,
                                       self.nbr_t)])
            c.num_segments = self.nseg
            c.segment_nodes_dev = self.counts.data_ptr()
            self._cstruct = c
        return c


class _Captured:
    def __init__(self, graph: StagedPairGraph, cuda_graph, keep=()):
        self.graph = graph
        self.cuda_graph = cuda_graph
        # what the graph writes or reads across replays and does not own:
        # the weight images it regenerates, the reducer events it waits on
        self.keep = list(keep)


def _drain_collectives(*groups) -> None:
    """Before a capture: wait until the process groups' outstanding (eager)
    collectives are retired from their watchdog's work list.  The RCCL
    watchdog thread polls the events of those works; a poll that lands inside
    the capture window intermittently aborted the process (measured: the
    captured data-parallel test aborted in 2 of 4 runs without this)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    seen = set()
    for g in (*groups, dist.group.WORLD):
        if g is None or id(g) in seen:
            continue
        seen.add(id(g))
        wait = getattr(g, "_wait_for_pending_works", None)
        if wait is not None:
            wait()


class CapturedTrainStep:
    """``step(xis, xjs) -> loss``: one MolCLR training step (molclr.py:108-128:
    zero_grad, the paired encoder pass, normalize, NT-Xent, backward, Adam)
    replayed from a HIP graph captured per capacity bucket.

    Lookup is by capacity, not by exact size: a batch pair runs on the
    smallest captured graph whose node / edge capacities hold it (same
    graphs per view), provided the node padding stays within ``node_slack``
    rows of the batch's own rounded size -- padding rows cost GEMM / BatchNorm
    / aggregation time, padding edge slots almost nothing.  Otherwise a new
    graph is captured at the batch's node count rounded up to
    ``node_quantum`` and its edge count plus ``edge_headroom`` rounded up to
    ``edge_quantum``.  Over an epoch the set of captures converges to a short
    ladder covering the batch-size spread (a handful of graphs at B = 512);
    ``prepare(pairs)`` captures what a known set of batches needs ahead of
    time.

    Memory: every capture gets its OWN graph memory pool (a c2 bucket holds
    ~1.5 GB of arena and workspace; a few buckets are a few percent of the
    288 GB HBM), so no capture can hand another capture's blocks to a third
    party, whatever order graphs replay in.  Cross-replay state lives outside
    every pool (parameters, gradients, Adam moments, BatchNorm running
    statistics, the loss and status buffers below, the staging buffers, the
    weight images -- ops.weight_planes never allocates an image inside a
    capture).  tests/test_gpu_graph_step.py alternates buckets against eager
    steps and checks that no step reads memory it did not write
    (test_no_uninitialised_reads).

    The returned loss tensor is this object's own buffer, overwritten by the
    next step.  ``status`` ORs every replayed batch's input-validity word
    (sticky: ``check()`` raises for an invalid batch at any earlier step).
    Requirements: a model with the paired executor path (``forward_staged``),
    a FusedAdam optimizer.  Data parallel: a criterion with a process group,
    and (optionally) an OverlappedGradReducer over the same optimizer --
    without one, the flat gradient is all-reduced in one collective.  The
    process group's communicator must exist before the first capture (any
    collective, e.g. the initial parameter broadcast, creates it)."""

    def __init__(self, model, optimizer, criterion, node_quantum: int = 256,
                 edge_quantum: int = 2048, max_graphs: int = 16, node_slack: int | None = None,
                 edge_headroom: float = 0.04, reducer=None):
        from .optim import FusedAdam
        if not isinstance(optimizer, FusedAdam):
            raise TypeError("CapturedTrainStep needs molclr_amd.optim.FusedAdam "
                            "(learning rate and step counter on the device)")
        if not hasattr(model, "forward_staged"):
            raise TypeError("CapturedTrainStep: the model has no forward_staged")
        self.group = getattr(criterion, "group", None)
        if reducer is not None and reducer.flat is not optimizer.flat_grad:
            raise ValueError("CapturedTrainStep: the reducer must reduce this optimizer's gradients")
        self.reducer = reducer
        self.model, self.optimizer, self.criterion = model, optimizer, criterion
        self.node_quantum, self.edge_quantum = int(node_quantum), int(edge_quantum)
        self.node_slack = 2 * self.node_quantum if node_slack is None else int(node_slack)
        self.edge_headroom = float(edge_headroom)
        self.max_graphs = int(max_graphs)
        self.device = optimizer.flat.device
        self._graphs: OrderedDict = OrderedDict()
        self.loss = torch.zeros((), dtype=torch.float32, device=self.device)
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.captures = 0
        self.replays = 0
        self.eager_steps = 0  # data parallel: batches no captured graph held
        self._one = None
        self.last_graph: StagedPairGraph | None = None

    @staticmethod
    def _need(xis, xjs) -> tuple:
        n = int(xis.x.shape[0]) + int(xjs.x.shape[0])
        e = int(xis.edge_index.shape[1]) + int(xjs.edge_index.shape[1])
        return n, e, _num_graphs_of(xis), _num_graphs_of(xjs)

    def bucket(self, xis, xjs) -> tuple:
        """(node_cap, edge_cap, G_i, G_j) a new capture for this pair gets."""
        n, e, gi, gj = self._need(xis, xjs)
        e_cap = _round_up(int(e * (1.0 + self.edge_headroom)) + 1, self.edge_quantum)
        return (_round_up(n, self.node_quantum), e_cap, gi, gj)

    def lookup(self, xis, xjs):
        """The captured entry this pair would replay on, or None."""
        n, e, gi, gj = self._need(xis, xjs)
        limit = _round_up(n, self.node_quantum) + self.node_slack
        best = None
        for ent in self._graphs.values():
            g = ent.graph
            if (g.num_nodes >= n and g.num_edges >= e and g.num_nodes <= limit
                    and g.graphs_per_segment == [gi, gj]):
                if best is None or (g.num_nodes, g.num_edges) < (best.graph.num_nodes,
                                                                 best.graph.num_edges):
                    best = ent
        return best

    def _capture(self, key, pair=None) -> _Captured:
        """Capture a graph of capacities ``key``; ``pair`` (if given) is staged
        into it first (the capture itself records, it runs nothing)."""
        if not self.model._executor_ok() or self.model._dim_pad():
            raise NotImplementedError(
                "CapturedTrainStep: the model must run through the encoder executor with "
                "emb_dim a multiple of the kernels' width (dropout 0, tracked BatchNorm)")
        ops._check_no_timer()
        graph = StagedPairGraph(self.device, key[0], key[1], key[2:])
        if pair is not None:
            graph.stage(list(pair))
        opt = self.optimizer
        opt.sync_lr()
        # the capture must record the weight-plane regeneration: make every
        # cached image stale so the forward's first lookup refreshes them all
        ops.bump_param_generation()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        _drain_collectives(self.group, getattr(self.reducer, "group", None))
        # data parallel: the process group's watchdog thread polls its events
        # while we capture; thread-local capture keeps those calls legal
        mode = "global" if self.group is None else "thread_local"
        self._dry_run(graph)
        ops.CAPTURE_SCOPE = {id(p) for p in self.model.parameters()}
        ops.CAPTURE_KEEP = keep = []
        try:
            self._record(g, mode, graph, opt)
        finally:
            ops.CAPTURE_SCOPE = None
            ops.CAPTURE_KEEP = None
        if self.reducer is not None:
            keep += self.reducer.capture_events
        self.captures += 1
        # a capture only records: the cached images must be regenerated by
        # the next eager use as well
        ops.bump_param_generation()
        return _Captured(graph, g, keep)

    def _dry_run(self, graph):
        """The step's forward and backward through the Python layer with every
        library call skipped (nothing runs on the GPU; the process group's
        NT-Xent gathers do run, on every rank alike: captures are made in
        lockstep).  What it leaves behind is what the capture must not
        allocate from its pool: the weight images the step reads, created
        here from the ordinary allocator (regenerated inside the graph)."""
        from . import _lib
        if self._one is None:  # d loss / d loss, outside every pool
            self._one = torch.ones((), dtype=torch.float32, device=self.device)
        with _lib.dry_run():
            _, z = self.model.forward_staged(graph)
            loss = self.criterion.forward_pair_normalized(z)
            loss.backward(self._one)
        del loss, z
        # the images it created hold nothing yet: the capture must record
        # their regeneration
        ops.bump_param_generation()
        torch.cuda.synchronize(self.device)

    def _record(self, g, mode, graph, opt):
        """The step's work into g (the tensors it allocates live in the pool)."""
        # a private pool per capture (see the class docstring)
        with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle(), capture_error_mode=mode):
            graph.build()
            opt.zero_grad()
            if self.reducer is not None:
                self.reducer.arm()
            _, z = self.model.forward_staged(graph)
            loss = self.criterion.forward_pair_normalized(z)
            # the seed gradient from a tensor made before the capture: no
            # fill kernel in the graph for autograd's ones_like(loss)
            loss.backward(self._one)
            if self.reducer is not None:  # bucketed, overlapped with the backward
                self.reducer.finish()
            elif self.group is not None:
                from .distributed import allreduce_grads
                allreduce_grads(opt.flat_grad, self.group)
            opt.step(sync_lr=False, tick=False)
            # one closing launch: Adam's step counter, the loss into this
            # object's buffer, the batch's validity bits (written by the graph
            # build and the atom embedding) into the sticky status word
            _lib.call("molclr_step_tail", opt._step_dev.data_ptr(), loss.data_ptr(),
                      self.loss.data_ptr(), graph.status.data_ptr(), self.status.data_ptr(),
                      _lib.stream_of(self.device))
        del loss, z

    def _insert(self, ent) -> None:
        self._graphs[id(ent)] = ent
        if len(self._graphs) > self.max_graphs:
            self._graphs.popitem(last=False)

    def _entry(self, xis, xjs):
        ent = self.lookup(xis, xjs)
        if ent is None:
            ent = self._capture(self.bucket(xis, xjs), (xis, xjs))  # stages this batch too
            self._insert(ent)
            return ent, True
        if not self._multi_rank():
            # one process: least-recently-replayed eviction.  Several ranks
            # replay different buckets, so a replay must not reorder the set:
            # captures (prepare / prepare_sizes) are inserted in lockstep and
            # evicted in capture order, leaving every rank the same graphs
            # and the same lookup() decisions
            self._graphs.move_to_end(id(ent))
        return ent, False

    # -- data parallel: captures in lockstep ----------------------------------
    def _multi_rank(self) -> bool:
        import torch.distributed as dist
        return (self.group is not None and dist.is_available() and dist.is_initialized()
                and dist.get_world_size(self.group) > 1)

    def _global_sizes(self, sizes) -> list:
        """Every rank's (nodes, edges) sizes (one all-gather of a padded list),
        so that all ranks capture the same buckets in the same order."""
        import torch.distributed as dist
        loc = torch.tensor([[int(a), int(b)] for a, b in sizes] or [[0, 0]],
                           dtype=torch.long, device=self.device)[: max(len(sizes), 1)]
        n = torch.tensor([len(sizes)], dtype=torch.long, device=self.device)
        ns = [torch.zeros_like(n) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(ns, n, group=self.group)
        most = max(1, max(int(t.item()) for t in ns))
        pad = torch.zeros(most, 2, dtype=torch.long, device=self.device)
        pad[: loc.shape[0]] = loc
        outs = [torch.zeros_like(pad) for _ in ns]
        dist.all_gather(outs, pad, group=self.group)
        return sorted({(int(a), int(b)) for o, k in zip(outs, ns)
                       for a, b in o[: int(k.item())].tolist()}, reverse=True)

    def prepare(self, pairs) -> int:
        """Capture (without running) every graph the given batch pairs need;
        returns the number of new captures.  Data parallel over several ranks:
        the union of every rank's sizes is captured on every rank, in the same
        order (a collective: all ranks call it together)."""
        before = self.captures
        pairs = list(pairs)
        if self._multi_rank():
            sizes = [self._need(a, b)[:2] for a, b in pairs]
            gi = {self._need(a, b)[2] for a, b in pairs}
            gj = {self._need(a, b)[3] for a, b in pairs}
            if len(gi) != 1 or len(gj) != 1:
                raise ValueError("CapturedTrainStep.prepare: data parallel batches must hold a "
                                 "fixed number of molecules per view")
            return self.prepare_sizes(sizes, gi.pop(), gj.pop())
        for xis, xjs in pairs:
            self._entry(xis, xjs)
        return self.captures - before

    def prepare_sizes(self, sizes, graphs_i: int, graphs_j: int) -> int:
        """Capture what batches of the given (nodes, edges) sizes -- both views
        together, ``graphs_i`` / ``graphs_j`` molecules per view -- will need,
        largest first, so that each capture serves every smaller size within
        the node slack (captures spaced ~node_slack + node_quantum apart).
        Nothing is staged: the first replay stages its batch.  Returns the
        number of new captures.  Data parallel over several ranks: a
        collective (every rank captures the union of all ranks' sizes)."""
        before = self.captures
        if self._multi_rank():
            sizes = self._global_sizes(list(sizes))

        class _V:  # the shape view lookup() / bucket() read
            def __init__(self, n, e, g):
                self.x = torch.empty(n, 0)
                self.edge_index = torch.empty(2, e)
                self._num_graphs = g

            @property
            def num_graphs(self):
                return self._num_graphs

        for n, e in sorted(((int(a), int(b)) for a, b in sizes), reverse=True):
            vi, vj = _V(n, e, graphs_i), _V(0, 0, graphs_j)
            if self.lookup(vi, vj) is None:
                self._insert(self._capture(self.bucket(vi, vj)))
        return self.captures - before

    def _eager(self, xis, xjs) -> torch.Tensor:
        """The same step without a graph (a data-parallel batch no captured
        graph holds): the same collectives in the same order as a replay, so
        ranks replaying graphs and a rank stepping eagerly stay matched."""
        from .data import pair_graph
        opt = self.optimizer
        opt.zero_grad()
        if self.reducer is not None:
            self.reducer.arm()
        _, z = self.model.forward_pair(xis, xjs)
        loss = self.criterion.forward_pair_normalized(z)
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish()
        else:
            from .distributed import allreduce_grads
            allreduce_grads(opt.flat_grad, self.group)
        opt.step()
        self.loss.copy_(loss.detach())
        torch.bitwise_or(self.status, pair_graph(xis, xjs).status, out=self.status)
        self.eager_steps += 1
        self.last_graph = None
        return self.loss

    def __call__(self, xis, xjs) -> torch.Tensor:
        if self._multi_rank() and self.lookup(xis, xjs) is None:
            # capturing here would capture on this rank alone: step eagerly
            # (prepare / prepare_sizes capture in lockstep ahead of time)
            return self._eager(xis, xjs)
        ent, fresh = self._entry(xis, xjs)
        if not fresh:
            ent.graph.stage([xis, xjs])
            self.optimizer.sync_lr()
        ent.cuda_graph.replay()
        self.replays += 1
        # the replay's Adam step changed the weights behind Python's back
        ops.bump_param_generation()
        self.last_graph = ent.graph
        return self.loss

    # -- parity of the replayed step against the eager one ---------------------
    def _state(self):
        opt = self.optimizer
        bns = [b for b in getattr(self.model, "batch_norms", [])]
        return ([t.clone() for t in (opt.flat, opt.exp_avg, opt.exp_avg_sq, opt._step_dev)],
                [(b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone())
                 for b in bns])

    def _restore(self, state):
        opt = self.optimizer
        flat, bn = state
        with torch.no_grad():
            for dst, src in zip((opt.flat, opt.exp_avg, opt.exp_avg_sq, opt._step_dev), flat):
                dst.copy_(src)
            for b, (m, v, n) in zip(self.model.batch_norms, bn):
                b.running_mean.copy_(m)
                b.running_var.copy_(v)
                b.num_batches_tracked.copy_(n)
        ops.bump_param_generation()

    def replay_vs_eager(self, xis, xjs) -> dict:
        """One training step on (xis, xjs) run twice from the same state: the
        eager step (the library's launches issued from the host, the batch at
        its own size) and the replay of the captured graph that holds the
        batch (capacity buckets: padding rows past the batch).  Returns the
        differences -- loss, flat gradient and per parameter (norm-wise), the
        BatchNorm running statistics and the parameters after Adam -- and
        leaves the model where the replay took it.  molclr.py:107-128 is the
        step; tests/test_gpu_bench_parity.py holds these to 1e-6 (loss) /
        1e-5 (fp32 gradients) and bench.py records one in its line."""
        def rel(a, b):
            d = (a.double() - b.double()).norm().item()
            n = b.double().norm().item()
            return d / n if n > 0 else d

        opt = self.optimizer
        if self.lookup(xis, xjs) is None and self._multi_rank():
            raise RuntimeError("replay_vs_eager: no captured graph holds this batch")
        start = self._state()
        eager_before = self.eager_steps
        loss_e = self._eager(xis, xjs).clone()
        self.eager_steps = eager_before
        grad_e = opt.flat_grad.clone()
        after_e = self._state()
        self._restore(start)
        ent = self.lookup(xis, xjs)
        loss_r = self(xis, xjs).clone()
        ent = ent or self.lookup(xis, xjs)
        grad_r = opt.flat_grad.clone()
        after_r = self._state()
        torch.cuda.synchronize(self.device)
        names = {id(q): k for k, q in self.model.named_parameters()}
        per = {names[id(p)]: rel(grad_r[off:off + n], grad_e[off:off + n])
               for p, off, n in opt.views}
        # the bias feeding each BatchNorm has an exact gradient of 0 (the
        # BatchNorm removes the column mean): rounding noise in either path
        real = {k: v for k, v in per.items()
                if not (k.endswith("mlp.2.bias")
                        or (k.startswith("gnns.") and k.count(".") == 2 and k.endswith(".bias")))}
        worst = max(real, key=real.get)
        bn_rel = max([rel(a[0], b[0]) for a, b in zip(after_r[1], after_e[1])] +
                     [rel(a[1], b[1]) for a, b in zip(after_r[1], after_e[1])] or [0.0])
        n_nodes = int(xis.x.shape[0]) + int(xjs.x.shape[0])
        return {"loss_eager": float(loss_e.item()), "loss_replay": float(loss_r.item()),
                "loss_rel": abs(loss_r.item() - loss_e.item()) / max(abs(loss_e.item()), 1e-30),
                "grad_rel": rel(grad_r, grad_e),
                "grad_rel_worst_param": [worst, real[worst]],
                "running_stats_rel": bn_rel,
                "params_rel": rel(after_r[0][0], after_e[0][0]),
                "nodes": n_nodes, "node_capacity": int(ent.graph.num_nodes),
                "padding_rows": int(ent.graph.num_nodes) - n_nodes}

    @property
    def buckets(self) -> list:
        """(node_cap, edge_cap) of every live capture."""
        return [(e.graph.num_nodes, e.graph.num_edges) for e in self._graphs.values()]

    def check(self) -> None:
        """Raise ValueError if any replayed batch so far had invalid inputs."""
        from .data import raise_for_status
        raise_for_status(int(self.status.item()))

    def close(self) -> None:
        """Release every captured graph (and the pool's memory) now.  Graphs
        holding RCCL collectives must go before their process group is
        destroyed: call this ahead of torch.distributed.destroy_process_group()."""
        torch.cuda.synchronize(self.device)
        self._graphs.clear()
        self.last_graph = None
        import gc
        gc.collect()
        torch.cuda.synchronize(self.device)
