"""Batched-graph data parallelism (one process per GPU, RCCL over xGMI).

The reference is single-device (molclr.py:45-53).  Scaling it out needs only
two exchanges per step, both chosen for a point-to-point xGMI fabric:

1. NT-Xent over the GLOBAL contrastive batch (molclr_amd.ops._NTXent):
   one all-gather of each rank's normalised rows [zj_local; zi_local]
   ([2 B_local, C]) reordered into the reference's [zj_all; zi_all]
   (gather_rows), and one of the per-row logsumexp with the rank's loss
   share appended (gather_lse_and_sum).  Because the NT-Xent weight matrix
   W_rc = P_rc + P_cr - 2[c = p(r)] is symmetric, each rank then computes the
   exact gradient of its own rows locally: no column-gradient reduce-scatter.
2. The SUM all-reduce of the flat gradient buffer (FusedAdam.flat_grad,
   ~9.6 MB fp32 for GIN 5x300).  OverlappedGradReducer splits it into a few
   large buckets in the order the backward finishes them -- projection heads,
   encoder layers L-1 .. 0, atom embeddings (one ~1.9 MB bucket per GIN
   layer, not per-parameter buckets: a ring over 7 xGMI links wants few,
   large collectives) -- and starts each on a side stream as soon as the
   encoder executor records that its gradients are final, so all but the
   last bucket's reduction hides behind the remaining backward.
   allreduce_grads is the single blocking collective (two-call steps).

BatchNorm statistics stay per rank and per view (the reference computes
them per forward call; like DDP without SyncBN), so an N-rank run is the
weak-scaling analogue of the single-GPU step, not bit-identical to a
single-GPU run at the global batch.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return rank, world, local


def init(backend: str | None = None) -> tuple[int, int, torch.device]:
    """Initialise the default process group when WORLD_SIZE > 1.

    Returns (rank, world_size, device); backend defaults to "nccl" (RCCL) on
    GPUs and "gloo" on CPU (MOLCLR_DIST_BACKEND overrides it: "gloo" lets
    several ranks share one GPU, as the multi-process GPU test does).
    """
    rank, world, local = env_world()
    if torch.cuda.is_available():
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        be = backend or os.environ.get("MOLCLR_DIST_BACKEND") or (
            "nccl" if device.type == "cuda" else "gloo")
        kw = dict(backend=be, rank=rank, world_size=world)
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world, device


def graph_capturable() -> bool:
    """Whether a HIP graph can hold the step's collectives: RCCL ("nccl")
    enqueues them on the stream, gloo runs them on the host (no process group:
    nothing to capture)."""
    return not (dist.is_available() and dist.is_initialized()) or dist.get_backend() == "nccl"


def _all_gather_stack(t: torch.Tensor, group=None) -> torch.Tensor:
    """[world, *t.shape]: every rank's t, in rank order.  One collective
    (all_gather_into_tensor on RCCL; the list form on backends without it)."""
    world = dist.get_world_size(group)
    t = t.contiguous()
    out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, t, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), t, group=group)
    return out


def gather_rows(local_rows: torch.Tensor, group=None) -> torch.Tensor:
    """Rows [zj_local; zi_local] ([2 B_l, C]) of every rank -> the global
    R = [zj_all; zi_all] ([2 B, C], B = world * B_l) of utils/nt_xent.py:48,
    rank r's molecules at [r B_l, (r+1) B_l) of each half."""
    g = _all_gather_stack(local_rows, group)          # [W, 2 B_l, C]
    W, two_bl = g.shape[0], g.shape[1]
    bl = two_bl // 2
    return torch.cat([g[:, :bl].reshape(W * bl, -1), g[:, bl:].reshape(W * bl, -1)], 0)


def gather_lse(local_lse: torch.Tensor, group=None) -> torch.Tensor:
    """Per-row logsumexp [2 B_l] of every rank -> [2 B] in R's row order."""
    g = _all_gather_stack(local_lse, group)            # [W, 2 B_l]
    bl = g.shape[1] // 2
    return torch.cat([g[:, :bl].reshape(-1), g[:, bl:].reshape(-1)], 0)


def gather_lse_and_sum(local_lse: torch.Tensor, local_sum: torch.Tensor, group=None):
    """gather_lse and the SUM of a per-rank scalar (the loss share) in one
    all-gather: ([2 B] lse in R's row order, Σ_ranks local_sum in rank order
    -- the same value on every rank)."""
    n = local_lse.shape[0]
    g = _all_gather_stack(torch.cat([local_lse, local_sum.reshape(1).to(local_lse.dtype)]), group)
    bl = n // 2
    lse = torch.cat([g[:, :bl].reshape(-1), g[:, bl:n].reshape(-1)], 0)
    return lse, g[:, n].sum()


def global_row_index(b_local: int, rank: int, world: int, device) -> torch.Tensor:
    """Global R row of each local row [zj_local; zi_local] (int32 [2 B_l])."""
    B = b_local * world
    base = torch.arange(b_local, dtype=torch.int32, device=device) + rank * b_local
    return torch.cat([base, base + B])


def allreduce_grads(flat_grad: torch.Tensor, group=None) -> None:
    """SUM the flat gradient buffer over ranks (the loss already carries the
    global 1/2B normalisation, so the sum is the exact global gradient)."""
    from . import ops
    ops.join_side()  # side-stream weight gradients land in flat_grad
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)


def broadcast_params(flat: torch.Tensor, src: int = 0, group=None) -> None:
    """Start every rank from rank 0's weights."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)


def max_over_ranks(value: float, device) -> float:
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([value], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return value


# ---------------------------------------------------------------------------
# Bucketed, overlapped gradient all-reduce
# ---------------------------------------------------------------------------
def gradient_buckets(model) -> list[list[torch.nn.Parameter]]:
    """The model's parameters grouped in the order the backward finalises
    them: the projection heads (feat_lin, out_lin), then encoder layer
    L-1 .. 0 (its convolution and BatchNorm), then the atom embeddings."""
    named = dict(model.named_parameters())
    L = model.num_layer
    heads = [p for n, p in named.items() if n.startswith(("feat_lin.", "out_lin."))]
    layers = [[p for n, p in named.items()
               if n.startswith((f"gnns.{l}.", f"batch_norms.{l}."))] for l in range(L - 1, -1, -1)]
    emb = [p for n, p in named.items() if n.startswith(("x_embedding1.", "x_embedding2."))]
    buckets = [heads, *layers, emb]
    if sum(len(b) for b in buckets) != len(named):
        raise ValueError("gradient_buckets: parameters outside the head / layer / embedding groups")
    return buckets


def bucketed_parameters(model) -> list[torch.nn.Parameter]:
    """Parameter order for FusedAdam that makes every gradient bucket one
    contiguous slice of its flat gradient buffer (the update rule is
    elementwise: the order changes nothing else)."""
    return [p for b in gradient_buckets(model) for p in b]


class OverlappedGradReducer:
    """SUM all-reduce of FusedAdam.flat_grad in gradient_buckets order,
    overlapped with the backward.

    ``arm()`` before the backward installs it as molclr_amd.ops' gradient
    hook: when the encoder's backward starts (the heads' gradients are
    final) the heads bucket is reduced; the encoder executor records one
    event per layer and one after the atom embeddings (molclr_*_encoder_grads
    .layer_done / .embed_done), and each layer's bucket is reduced behind its
    event on a side stream.  ``finish()`` makes the compute stream wait for
    every bucket before the optimizer step.  One encoder backward per step
    (the paired-view step); a second one would add to buckets already in
    flight and is refused."""

    def __init__(self, model, opt, group=None):
        self.group = group
        self.flat = opt.flat_grad
        off = {id(p): (o, (n + 3) // 4 * 4) for p, o, n in opt.views}  # FusedAdam's 4-aligned slots
        self.slices = []
        for b in gradient_buckets(model):
            spans = sorted(off[id(p)] for p in b)
            for (o0, n0), (o1, _) in zip(spans, spans[1:]):
                if o1 != o0 + n0:
                    raise ValueError("OverlappedGradReducer: build FusedAdam over "
                                     "bucketed_parameters(model)")
            self.slices.append((spans[0][0], spans[-1][0] + spans[-1][1]))
        self.num_layer = model.num_layer
        self.cuda = self.flat.is_cuda
        self.works, self.calls = [], 0
        self._begin_ev = None
        # events of the step being captured (CapturedTrainStep keeps them with
        # its graph); eager steps reuse self.events
        self.capture_events: list = []
        if self.cuda:
            self.stream = torch.cuda.Stream(device=self.flat.device)
            # eager steps' events: never handed to a graph
            self.eager_events = self._new_events()
            self.events = self.eager_events

    def _new_events(self):
        # the executor re-records these; a first record creates the handles
        ev = [torch.cuda.Event() for _ in range(self.num_layer + 1)]
        for e in ev:
            e.record()
        return ev

    # -- step protocol --------------------------------------------------------
    def arm(self):
        from . import ops
        self.works, self.calls = [], 0
        if self.cuda and torch.cuda.is_current_stream_capturing():
            # every capture records and waits on events of its own: no event
            # handle is shared by two graphs
            self.events = self._new_events()
            self.capture_events = list(self.events)
        elif self.cuda:
            # an eager step (CapturedTrainStep._eager included) never
            # re-records the handles the last captured graph holds
            self.events = self.eager_events
        ops.set_grad_hook(self)

    def finish(self):
        from . import ops
        ops.set_grad_hook(None)
        ops.join_side()
        if self.calls == 0:  # no executor backward ran (per-op path): one collective
            allreduce_grads(self.flat, self.group)
            return
        for w in self.works:
            w.wait()  # the current stream waits for the bucket's collective
        self.works = []
        if self._begin_ev is not None:
            if torch.cuda.is_current_stream_capturing():
                self.capture_events.append(self._begin_ev)
            self._begin_ev = None

    def _reduce(self, i, after=None):
        lo, hi = self.slices[i]
        view = self.flat[lo:hi]
        if not self.cuda:
            dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group)
            return
        with torch.cuda.stream(self.stream):
            if after is not None:
                self.stream.wait_event(after)
            self.works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True))

    # -- hooks called by molclr_amd.ops' encoder backward ----------------------
    def encoder_backward_begin(self):
        if self.calls:
            raise RuntimeError("OverlappedGradReducer: one encoder backward per step (paired views)")
        self.calls += 1
        if self.cuda:
            # kept until finish(): the side stream's wait must not outlive it
            self._begin_ev = ev = torch.cuda.Event()
            ev.record()
            self._reduce(0, ev)
        else:
            self._reduce(0)

    def layer_event_handles(self):
        """[layer 0 .. L-1, embeddings] hipEvent_t handles for the executor."""
        if not self.cuda:
            return None
        return [e.cuda_event for e in self.events]

    def encoder_backward_enqueued(self):
        L = self.num_layer
        for k, l in enumerate(range(L - 1, -1, -1)):
            self._reduce(1 + k, self.events[l] if self.cuda else None)
        self._reduce(1 + L, self.events[L] if self.cuda else None)
