"""``torch.ops.molclr.*``: the operator seam of SURVEY.md §8(b).

The reference's hot path calls PyG's ``MessagePassing.propagate`` /
``global_mean_pool`` and its own NT-Xent (models/ginet_molclr.py:29-44,113;
utils/nt_xent.py:47-65).  The same computations are registered here as torch
operators in the ``molclr`` namespace (``torch.library.custom_op``), each
with its backward (``register_autograd``) and a shape function
(``register_fake``), so that TorchScript-free graph tools (``torch.compile``,
``torch.library`` users, ``torch.fx``) see them as ops rather than opaque
Python.  The kernels are the C ABI's (include/molclr.h) -- the same launches
molclr_amd.ops' autograd functions issue, so results are bit-identical to
them; ``import molclr_amd.torch_ops`` registers the set:

=======================================  =====================================
op                                       reference
=======================================  =====================================
graph_build(edge_index, edge_attr,       PyG collate + add_self_loops
  batch, num_nodes, num_graphs)          (ginet_molclr.py:31-37)
gine_aggregate(h, E1, E2, graph...)      GINEConv.propagate (:29-44)
gine_aggregate_bwd(...)                  its backward (dh, dE1, dE2)
segment_pool(h, graph_ptr, mode)         global_mean_pool / global_add_pool (:113)
segment_pool_bwd(...)                    its backward
l2_normalize(z, eps)                     F.normalize (molclr.py:63-64)
l2_normalize_bwd(...)                    its backward
nt_xent(zis, zjs, batch_size, T, cos)    NTXentLoss.forward (nt_xent.py:47-65)
nt_xent_bwd(...)                         its backward (dzis, dzjs)
=======================================  =====================================

The graph tensors of the aggregation ops are graph_build's outputs in its
order: (rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount, graph_ptr,
status).  Missing library => ImportError; a CPU tensor => RuntimeError (the
ops are registered for CUDA/HIP only).
"""
from __future__ import annotations

import torch
from torch.library import custom_op

from . import _lib, ops
from .data import DeviceGraph, raise_for_status  # noqa: F401  (re-exported for callers)

_lib.load()  # fail at import, not at the first call, when the library is missing

_GRAPH_FIELDS = ("rowptr", "col", "ecode", "rowptr_t", "col_t", "nbr", "nbr_t", "ecount",
                 "graph_ptr", "status")


def _cuda(*ts):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("torch.ops.molclr runs on the GPU only; got a %s tensor" % t.device)


def _stream(t):
    return _lib.stream_of(t.device)


# ---------------------------------------------------------------------------
# graph build
# ---------------------------------------------------------------------------
@custom_op("molclr::graph_build", mutates_args=(), device_types="cuda")
def graph_build(edge_index: torch.Tensor, edge_attr: torch.Tensor, batch: torch.Tensor,
                num_nodes: int, num_graphs: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                                          torch.Tensor, torch.Tensor, torch.Tensor,
                                                          torch.Tensor, torch.Tensor, torch.Tensor,
                                                          torch.Tensor]:
    """Destination CSR (stable by destination, the implicit self loop last),
    source CSC, neighbour slots, bond-type counts and graph offsets of one
    collated batch (molclr_graph_build)."""
    _cuda(edge_index, edge_attr, batch)
    g = DeviceGraph(edge_index, edge_attr, int(num_nodes), batch, int(num_graphs))
    return tuple(getattr(g, f) for f in _GRAPH_FIELDS)


@graph_build.register_fake
def _(edge_index, edge_attr, batch, num_nodes, num_graphs):
    E = edge_index.shape[1]
    N = num_nodes
    i32 = dict(dtype=torch.int32, device=edge_index.device)
    e = max(E, 1)
    n = max(N, 1)
    return (edge_index.new_empty(N + 1, **i32), edge_index.new_empty(e, **i32),
            edge_index.new_empty(e, dtype=torch.uint8), edge_index.new_empty(N + 1, **i32),
            edge_index.new_empty(e, **i32), edge_index.new_empty(4 * n, **i32),
            edge_index.new_empty(4 * n, **i32), edge_index.new_empty(8 * n, **i32),
            edge_index.new_empty(num_graphs + 1, **i32), edge_index.new_empty(1, **i32))


# ---------------------------------------------------------------------------
# GINE aggregation
# ---------------------------------------------------------------------------
def _check_graph(N, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount):
    """Host-side shape / dtype checks of graph_build's tensors against N rows
    (a mismatched tensor would send the kernels' index reads out of bounds)."""
    i32 = torch.int32
    E = col.shape[0]
    want = ((rowptr, (N + 1,), i32), (rowptr_t, (N + 1,), i32), (col, (E,), i32),
            (col_t, (E,), i32), (ecode, (E,), torch.uint8), (nbr, (4 * max(N, 1),), i32),
            (nbr_t, (4 * max(N, 1),), i32), (ecount, (8 * max(N, 1),), i32))
    for k, (t, shape, dt) in enumerate(want):
        if tuple(t.shape) != shape or t.dtype != dt or not t.is_cuda:
            raise ValueError(f"molclr graph tensor {k}: {tuple(t.shape)} {t.dtype}, expected "
                             f"{shape} {dt} on the GPU (graph_build's outputs 0..7, in order)")


@custom_op("molclr::gine_aggregate", mutates_args=(), device_types="cuda")
def gine_aggregate(h: torch.Tensor, E1: torch.Tensor, E2: torch.Tensor, rowptr: torch.Tensor,
                   col: torch.Tensor, ecode: torch.Tensor, rowptr_t: torch.Tensor,
                   col_t: torch.Tensor, nbr: torch.Tensor, nbr_t: torch.Tensor,
                   ecount: torch.Tensor) -> torch.Tensor:
    """agg_i = Σ_{in-edges k of i, self loop last} (h[src_k] + E1[bt_k] + E2[bd_k]) in PyG's
    order (molclr_edge_tables_combine + molclr_gine_aggregate_fwd).  The graph
    tensors are graph_build's outputs 0..7 in its order (rowptr, col, ecode,
    rowptr_t, col_t, nbr, nbr_t, ecount); the source-CSC half is the backward's."""
    _cuda(h, E1, E2)
    h = h.contiguous()
    N, D = h.shape
    _check_graph(N, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount)
    Ec = ops.edge_tables_combine([E1], [E2])[0]
    out = torch.empty_like(h)
    _lib.call("molclr_gine_aggregate_fwd", h.data_ptr(), rowptr.data_ptr(), col.data_ptr(),
              ecode.data_ptr(), nbr.data_ptr(), Ec.data_ptr(), out.data_ptr(), N, D, _stream(h))
    return out


@gine_aggregate.register_fake
def _(h, E1, E2, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount):
    return torch.empty_like(h)


@custom_op("molclr::gine_aggregate_bwd", mutates_args=(), device_types="cuda")
def gine_aggregate_bwd(g: torch.Tensor, rowptr_t: torch.Tensor, col_t: torch.Tensor,
                       nbr_t: torch.Tensor, ecount: torch.Tensor, n_e1: int,
                       n_e2: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dh, dE1, dE2) of gine_aggregate (molclr_gine_aggregate_bwd: the
    transposed gather in index_select order, count-weighted table sums)."""
    g = g.contiguous()
    N, D = g.shape
    i32 = torch.int32
    for k, (t, shape) in enumerate(((rowptr_t, (N + 1,)), (nbr_t, (4 * max(N, 1),)),
                                    (ecount, (8 * max(N, 1),)))):
        if tuple(t.shape) != shape or t.dtype != i32:
            raise ValueError(f"gine_aggregate_bwd: graph tensor {k} {tuple(t.shape)} {t.dtype}, "
                             f"expected {shape} int32")
    if col_t.dtype != i32 or col_t.dim() != 1:
        raise ValueError("gine_aggregate_bwd: col_t must be int32 [E]")
    dh = torch.empty_like(g)
    dE1 = torch.zeros(n_e1, D, dtype=torch.float32, device=g.device)
    dE2 = torch.zeros(n_e2, D, dtype=torch.float32, device=g.device)
    wsb = ops._wsq("molclr_gine_aggregate_bwd_workspace_bytes", N, D)
    ws = ops._ws(wsb, g.device)
    _lib.call("molclr_gine_aggregate_bwd", g.data_ptr(), rowptr_t.data_ptr(), col_t.data_ptr(),
              nbr_t.data_ptr(), ecount.data_ptr(), dh.data_ptr(), dE1.data_ptr(), dE2.data_ptr(),
              N, D, 0, ws.data_ptr(), wsb, _stream(g))
    return dh, dE1, dE2


@gine_aggregate_bwd.register_fake
def _(g, rowptr_t, col_t, nbr_t, ecount, n_e1, n_e2):
    D = g.shape[1]
    return torch.empty_like(g), g.new_empty(n_e1, D), g.new_empty(n_e2, D)


# ---------------------------------------------------------------------------
# pooling
# ---------------------------------------------------------------------------
_POOL = {"mean": 0, "add": 1}


@custom_op("molclr::segment_pool", mutates_args=(), device_types="cuda")
def segment_pool(h: torch.Tensor, graph_ptr: torch.Tensor, mode: int) -> torch.Tensor:
    """global_mean_pool (mode 0) / global_add_pool (mode 1) over graph_ptr."""
    _cuda(h)
    h = h.contiguous()
    N, D = h.shape
    G = graph_ptr.shape[0] - 1
    out = torch.empty(G, D, dtype=torch.float32, device=h.device)
    _lib.call("molclr_segment_pool_fwd", h.data_ptr(), graph_ptr.data_ptr(), out.data_ptr(), G, D,
              int(mode), _stream(h))
    return out


@segment_pool.register_fake
def _(h, graph_ptr, mode):
    return h.new_empty(graph_ptr.shape[0] - 1, h.shape[1])


@custom_op("molclr::segment_pool_bwd", mutates_args=(), device_types="cuda")
def segment_pool_bwd(dout: torch.Tensor, graph_ptr: torch.Tensor, num_nodes: int,
                     mode: int) -> torch.Tensor:
    dout = dout.contiguous()
    G, D = dout.shape
    dh = torch.empty(num_nodes, D, dtype=torch.float32, device=dout.device)
    _lib.call("molclr_segment_pool_bwd", dout.data_ptr(), graph_ptr.data_ptr(), dh.data_ptr(),
              num_nodes, G, D, int(mode), _stream(dout))
    return dh


@segment_pool_bwd.register_fake
def _(dout, graph_ptr, num_nodes, mode):
    return dout.new_empty(num_nodes, dout.shape[1])


# ---------------------------------------------------------------------------
# F.normalize
# ---------------------------------------------------------------------------
@custom_op("molclr::l2_normalize", mutates_args=(), device_types="cuda")
def l2_normalize(z: torch.Tensor, eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """(y, |z| per row): F.normalize(z, dim=1, eps) (molclr_l2norm_fwd)."""
    _cuda(z)
    z = z.contiguous()
    rows, D = z.shape
    y = torch.empty_like(z)
    norm = torch.empty(rows, dtype=torch.float32, device=z.device)
    _lib.call("molclr_l2norm_fwd", z.data_ptr(), y.data_ptr(), norm.data_ptr(), rows, D,
              float(eps), _stream(z))
    return y, norm


@l2_normalize.register_fake
def _(z, eps):
    return torch.empty_like(z), z.new_empty(z.shape[0])


@custom_op("molclr::l2_normalize_bwd", mutates_args=(), device_types="cuda")
def l2_normalize_bwd(dy: torch.Tensor, y: torch.Tensor, norm: torch.Tensor,
                     eps: float) -> torch.Tensor:
    dy = dy.contiguous()
    rows, D = dy.shape
    dz = torch.empty_like(dy)
    _lib.call("molclr_l2norm_bwd", dy.data_ptr(), y.data_ptr(), norm.data_ptr(), dz.data_ptr(),
              rows, D, float(eps), _stream(dy))
    return dz


@l2_normalize_bwd.register_fake
def _(dy, y, norm, eps):
    return torch.empty_like(dy)


# ---------------------------------------------------------------------------
# NT-Xent (one process: batch_size = the rows' B)
# ---------------------------------------------------------------------------
@custom_op("molclr::nt_xent", mutates_args=(), device_types="cuda")
def nt_xent(zis: torch.Tensor, zjs: torch.Tensor, batch_size: int, temperature: float,
            use_cosine_similarity: bool) -> torch.Tensor:
    """NTXentLoss(device, batch_size, temperature, use_cosine_similarity)(zis, zjs)."""
    _cuda(zis, zjs)
    return ops.nt_xent(zis, zjs, batch_size, temperature, use_cosine_similarity).detach()


@nt_xent.register_fake
def _(zis, zjs, batch_size, temperature, use_cosine_similarity):
    return zis.new_empty(())


@custom_op("molclr::nt_xent_bwd", mutates_args=(), device_types="cuda")
def nt_xent_bwd(grad: torch.Tensor, zis: torch.Tensor, zjs: torch.Tensor, batch_size: int,
                temperature: float, use_cosine_similarity: bool
                ) -> tuple[torch.Tensor, torch.Tensor]:
    """(dzis, dzjs) of nt_xent for the upstream scalar ``grad`` (the row
    scaling and the forward's row logsumexp are recomputed: molclr_ntxent_prep,
    _fwd, _bwd, _prep_bwd)."""
    R = torch.cat([zjs, zis], 0).contiguous()
    n, C = R.shape
    B = n // 2
    if batch_size != B:
        raise ValueError(f"nt_xent_bwd: batch_size {batch_size} for {B} rows")
    dev, st, cos = R.device, _stream(R), int(use_cosine_similarity)
    rhat, norm = torch.empty_like(R), torch.empty(n, dtype=torch.float32, device=dev)
    _lib.call("molclr_ntxent_prep", R.data_ptr(), rhat.data_ptr(), norm.data_ptr(), n, C, cos, st)
    gidx = torch.arange(n, dtype=torch.int32, device=dev)
    lse, lr = torch.empty(n, device=dev), torch.empty(n, device=dev)
    wsb = ops._wsq("molclr_ntxent_workspace_bytes", n, n, C)
    ws = ops._ws(wsb, dev)
    _lib.call("molclr_ntxent_fwd_impl", rhat.data_ptr(), gidx.data_ptr(), rhat.data_ptr(), n, n, C,
              B, float(temperature), lse.data_ptr(), lr.data_ptr(), None, ws.data_ptr(), wsb, st, -1)
    g = grad.to(torch.float32).reshape(1).contiguous()
    drhat = torch.empty_like(rhat)
    _lib.call("molclr_ntxent_bwd_impl", rhat.data_ptr(), gidx.data_ptr(), rhat.data_ptr(),
              lse.data_ptr(), g.data_ptr(), n, n, C, B, float(temperature), None, drhat.data_ptr(),
              ws.data_ptr(), wsb, st, -1)
    dR = torch.empty_like(rhat)
    _lib.call("molclr_ntxent_prep_bwd", drhat.data_ptr(), rhat.data_ptr(), norm.data_ptr(),
              dR.data_ptr(), n, C, cos, st)
    return dR[B:].clone(), dR[:B].clone()


@nt_xent_bwd.register_fake
def _(grad, zis, zjs, batch_size, temperature, use_cosine_similarity):
    return torch.empty_like(zis), torch.empty_like(zjs)


# ---------------------------------------------------------------------------
# autograd
# ---------------------------------------------------------------------------
def _agg_setup(ctx, inputs, output):
    h, E1, E2, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount = inputs
    ctx.save_for_backward(rowptr_t, col_t, nbr_t, ecount)
    ctx.n = (E1.shape[0], E2.shape[0])


def _agg_backward(ctx, g):
    rowptr_t, col_t, nbr_t, ecount = ctx.saved_tensors
    dh, dE1, dE2 = torch.ops.molclr.gine_aggregate_bwd(g, rowptr_t, col_t, nbr_t, ecount, *ctx.n)
    return (dh, dE1, dE2) + (None,) * 8


gine_aggregate.register_autograd(_agg_backward, setup_context=_agg_setup)


def _pool_setup(ctx, inputs, output):
    h, graph_ptr, mode = inputs
    ctx.save_for_backward(graph_ptr)
    ctx.n, ctx.mode = h.shape[0], mode


def _pool_backward(ctx, dout):
    (graph_ptr,) = ctx.saved_tensors
    return torch.ops.molclr.segment_pool_bwd(dout, graph_ptr, ctx.n, ctx.mode), None, None


segment_pool.register_autograd(_pool_backward, setup_context=_pool_setup)


def _l2_setup(ctx, inputs, output):
    z, eps = inputs
    y, norm = output
    ctx.save_for_backward(y, norm)
    ctx.eps = eps


def _l2_backward(ctx, dy, dnorm):
    y, norm = ctx.saved_tensors
    return torch.ops.molclr.l2_normalize_bwd(dy, y, norm, ctx.eps), None


l2_normalize.register_autograd(_l2_backward, setup_context=_l2_setup)


def _ntx_setup(ctx, inputs, output):
    zis, zjs, batch_size, temperature, cos = inputs
    ctx.save_for_backward(zis, zjs)
    ctx.args = (batch_size, temperature, cos)


def _ntx_backward(ctx, grad):
    zis, zjs = ctx.saved_tensors
    da, db = torch.ops.molclr.nt_xent_bwd(grad, zis, zjs, *ctx.args)
    return da, db, None, None, None


nt_xent.register_autograd(_ntx_backward, setup_context=_ntx_setup)

OPS = ("graph_build", "gine_aggregate", "gine_aggregate_bwd", "segment_pool", "segment_pool_bwd",
       "l2_normalize", "l2_normalize_bwd", "nt_xent", "nt_xent_bwd")
