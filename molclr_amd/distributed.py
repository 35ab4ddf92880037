"""Batched-graph data parallelism (one process per GPU, RCCL over xGMI).

The reference is single-device (molclr.py:45-53).  Scaling it out needs only
two exchanges per step, both chosen for a point-to-point xGMI fabric:

1. NT-Xent over the GLOBAL contrastive batch (molclr_amd.ops._NTXent):
   one all-gather of each rank's normalised rows [zj_local; zi_local]
   ([2 B_local, C]) reordered into the reference's [zj_all; zi_all]
   (gather_rows), and one of the per-row logsumexp (gather_lse).  Because the NT-Xent weight matrix
   W_rc = P_rc + P_cr - 2[c = p(r)] is symmetric, each rank then computes the
   exact gradient of its own rows locally: no column-gradient reduce-scatter.
2. One SUM all-reduce of the flat gradient buffer (FusedAdam.flat_grad,
   ~9.6 MB fp32 for GIN 5x300) — a single large collective instead of
   per-parameter buckets, which is what a ring over 7 xGMI links wants.

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
    GPUs and "gloo" on CPU.
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
        be = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = dict(backend=be, rank=rank, world_size=world)
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world, device


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


def global_row_index(b_local: int, rank: int, world: int, device) -> torch.Tensor:
    """Global R row of each local row [zj_local; zi_local] (int32 [2 B_l])."""
    B = b_local * world
    base = torch.arange(b_local, dtype=torch.int32, device=device) + rank * b_local
    return torch.cat([base, base + B])


def allreduce_grads(flat_grad: torch.Tensor, group=None) -> None:
    """SUM the flat gradient buffer over ranks (the loss already carries the
    global 1/2B normalisation, so the sum is the exact global gradient)."""
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
