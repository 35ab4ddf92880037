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
gcn_aggregate(xw, E1, E2, bias, graph..) GCNConv.propagate + bias
                                         (gcn_molclr.py:72-91)
gcn_aggregate_bwd(...)                   its backward (dxw, dE1, dE2, dbias)
gcn_conv(x, W, bias, E1, E2, graph...)   GCNConv.forward (gcn_molclr.py:62-84):
                                         x @ W, then gcn_aggregate
gcn_conv_bwd(...)                        its backward
mlp(x, W1, b1, W2, b2)                   Linear -> ReLU -> Linear: GINEConv's
                                         update (ginet_molclr.py:19-23,46-47)
                                         and out_lin (:93-96)
mlp_bwd(...)                             its backward
linear(x, W, b)                          nn.Linear (feat_lin, :90-92)
linear_bwd(...)                          its backward
batch_norm_seg(z, gamma, beta, running   BatchNorm1d (+ ReLU) with one set of
  stats, seg_rows, training, momentum,   batch statistics per row segment
  eps, relu)                             (ginet_molclr.py:105-111; a segment
                                         per encoder call, molclr.py:57,60)
batch_norm_seg_bwd(...)                  its backward (dz, dgamma, dbeta)
=======================================  =====================================

GINEConv + BatchNorm (ginet_molclr.py:29-47,105-111) and GCNConv
(gcn_molclr.py:62-91) rebuilt on these ops alone: INTEGRATION.md §10.
These are Python ``torch.library.custom_op`` registrations over the C ABI,
not a C++ ``TORCH_LIBRARY`` block (SURVEY §8(b) proposed one): the kernels
are reached through ctypes (molclr_amd._lib), so no torch C++ extension has
to be built against the installed torch; the dispatcher sees the same ops.

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
    _cuda(g, rowptr_t, col_t, nbr_t, ecount)
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


def _check_ptr(graph_ptr, num_nodes, who):
    """graph_ptr as graph_build writes it: int32 [G+1] on the GPU, within the
    rows (PyG's int64 ``ptr`` would be read as int32: wrong segments and
    out-of-bounds reads).  The last entry is checked on the host."""
    _cuda(graph_ptr)
    if graph_ptr.dtype != torch.int32 or graph_ptr.dim() != 1 or graph_ptr.shape[0] < 1:
        raise ValueError(f"{who}: graph_ptr must be int32 [num_graphs + 1] (graph_build's "
                         f"output 8), got {graph_ptr.dtype} {tuple(graph_ptr.shape)}")
    if graph_ptr.shape[0] > 1:
        first, last = (int(v) for v in graph_ptr[[0, -1]].tolist())
        if first < 0 or last > num_nodes or last < first:
            raise ValueError(f"{who}: graph_ptr spans rows [{first}, {last}) of {num_nodes}")


@custom_op("molclr::segment_pool", mutates_args=(), device_types="cuda")
def segment_pool(h: torch.Tensor, graph_ptr: torch.Tensor, mode: int) -> torch.Tensor:
    """global_mean_pool (mode 0) / global_add_pool (mode 1) over graph_ptr."""
    _cuda(h)
    h = h.contiguous()
    if h.dtype != torch.float32 or h.dim() != 2:
        raise ValueError(f"segment_pool: h must be fp32 [N, D], got {h.dtype} {tuple(h.shape)}")
    if int(mode) not in (0, 1):
        raise ValueError(f"segment_pool: mode {mode} (0 = mean, 1 = add)")
    N, D = h.shape
    _check_ptr(graph_ptr, N, "segment_pool")
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
    _cuda(dout)
    dout = dout.contiguous().to(torch.float32)
    G, D = dout.shape
    _check_ptr(graph_ptr, int(num_nodes), "segment_pool_bwd")
    if graph_ptr.shape[0] != G + 1:
        raise ValueError(f"segment_pool_bwd: {G} graphs in dout, graph_ptr has "
                         f"{graph_ptr.shape[0]} entries")
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
    _cuda(dy, y, norm)
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
    _cuda(grad, zis, zjs)
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
# GCN aggregation / GCNConv
# ---------------------------------------------------------------------------
def _check_gcn_tables(E1, E2, bias, D):
    if tuple(E1.shape) != (5, 1) or tuple(E2.shape) != (3, 1):
        raise ValueError(f"GCN edge tables must be [5, 1] and [3, 1] (gcn_molclr.py:49-52), got "
                         f"{tuple(E1.shape)} {tuple(E2.shape)}")
    if tuple(bias.shape) != (D,):
        raise ValueError(f"GCN bias must be [{D}], got {tuple(bias.shape)}")


@custom_op("molclr::gcn_aggregate", mutates_args=(), device_types="cuda")
def gcn_aggregate(xw: torch.Tensor, E1: torch.Tensor, E2: torch.Tensor, bias: torch.Tensor,
                  rowptr: torch.Tensor, col: torch.Tensor, ecode: torch.Tensor,
                  rowptr_t: torch.Tensor, col_t: torch.Tensor, nbr: torch.Tensor,
                  nbr_t: torch.Tensor, ecount: torch.Tensor) -> torch.Tensor:
    """out_i = Σ_{in-edges k of i, self loop last} (xw[src_k] + E1[bt_k] + E2[bd_k]) + bias
    (GCNConv.propagate / message / update, gcn_molclr.py:79-91; its gcn_norm at
    :74 is discarded by the reference and not computed): molclr_gcn_aggregate_fwd."""
    _cuda(xw, E1, E2, bias)
    xw = xw.contiguous()
    N, D = xw.shape
    _check_graph(N, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount)
    _check_gcn_tables(E1, E2, bias, D)
    out = torch.empty_like(xw)
    _lib.call("molclr_gcn_aggregate_fwd", xw.data_ptr(), rowptr.data_ptr(), col.data_ptr(),
              ecode.data_ptr(), nbr.data_ptr(), E1.contiguous().data_ptr(),
              E2.contiguous().data_ptr(), bias.contiguous().data_ptr(), out.data_ptr(), N, D,
              _stream(xw))
    return out


@gcn_aggregate.register_fake
def _(xw, E1, E2, bias, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount):
    return torch.empty_like(xw)


@custom_op("molclr::gcn_aggregate_bwd", mutates_args=(), device_types="cuda")
def gcn_aggregate_bwd(g: torch.Tensor, rowptr_t: torch.Tensor, col_t: torch.Tensor,
                      nbr_t: torch.Tensor, ecount: torch.Tensor
                      ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dxw, dE1 [5,1], dE2 [3,1], dbias) of gcn_aggregate (molclr_gcn_aggregate_bwd)."""
    _cuda(g, rowptr_t, col_t, nbr_t, ecount)
    g = g.contiguous()
    N, D = g.shape
    i32 = torch.int32
    for k, (t, shape) in enumerate(((rowptr_t, (N + 1,)), (nbr_t, (4 * max(N, 1),)),
                                    (ecount, (8 * max(N, 1),)))):
        if tuple(t.shape) != shape or t.dtype != i32:
            raise ValueError(f"gcn_aggregate_bwd: graph tensor {k} {tuple(t.shape)} {t.dtype}, "
                             f"expected {shape} int32")
    dxw = torch.empty_like(g)
    f32 = dict(dtype=torch.float32, device=g.device)
    dE1, dE2, db = torch.empty(5, 1, **f32), torch.empty(3, 1, **f32), torch.empty(D, **f32)
    wsb = ops._wsq("molclr_gcn_aggregate_bwd_workspace_bytes", N, D)
    ws = ops._ws(wsb, g.device)
    _lib.call("molclr_gcn_aggregate_bwd", g.data_ptr(), rowptr_t.data_ptr(), col_t.data_ptr(),
              nbr_t.data_ptr(), ecount.data_ptr(), dxw.data_ptr(), dE1.data_ptr(), dE2.data_ptr(),
              db.data_ptr(), N, D, 0, ws.data_ptr(), wsb, _stream(g))
    return dxw, dE1, dE2, db


@gcn_aggregate_bwd.register_fake
def _(g, rowptr_t, col_t, nbr_t, ecount):
    D = g.shape[1]
    return torch.empty_like(g), g.new_empty(5, 1), g.new_empty(3, 1), g.new_empty(D)


class _Ctx:
    """The autograd context molclr_amd.ops' Functions expect, outside autograd:
    the seam ops below run those Functions' own forward / backward bodies (the
    same launches, so bit-identical results) and carry their saved state as
    extra op outputs.  Parameters are not FusedAdam-owned here: every gradient
    comes back as a fresh tensor."""

    def __init__(self, n_inputs):
        self.needs_input_grad = (True,) * n_inputs
        self.saved_tensors = ()

    def save_for_backward(self, *ts):
        self.saved_tensors = ts


def _graph_ns(rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount):
    import types
    return types.SimpleNamespace(rowptr=rowptr, col=col, ecode=ecode, rowptr_t=rowptr_t,
                                 col_t=col_t, nbr=nbr, nbr_t=nbr_t, ecount=ecount,
                                 num_edges=col.shape[0])


@custom_op("molclr::gcn_conv", mutates_args=(), device_types="cuda")
def gcn_conv(x: torch.Tensor, W: torch.Tensor, bias: torch.Tensor, E1: torch.Tensor,
             E2: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor, ecode: torch.Tensor,
             rowptr_t: torch.Tensor, col_t: torch.Tensor, nbr: torch.Tensor, nbr_t: torch.Tensor,
             ecount: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """GCNConv.forward (gcn_molclr.py:62-84): x @ W (W stored [in, out], :45,76),
    then gcn_aggregate.  Returns (out, xmax): xmax is max |x| for the h3 weight
    gradient (saved state, no gradient)."""
    _cuda(x, W, bias, E1, E2)
    _check_graph(x.shape[0], rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount)
    _check_gcn_tables(E1, E2, bias, W.shape[1])
    ctx = _Ctx(6)
    out = ops._GCNConv.forward(ctx, x, W, bias, E1, E2,
                               _graph_ns(rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount))
    xmax = ctx.xmax if ctx.h3 else x.new_empty(0)
    return out, xmax


@gcn_conv.register_fake
def _(x, W, bias, E1, E2, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount):
    return x.new_empty(x.shape[0], W.shape[1]), x.new_empty(0)


@custom_op("molclr::gcn_conv_bwd", mutates_args=(), device_types="cuda")
def gcn_conv_bwd(g: torch.Tensor, x: torch.Tensor, W: torch.Tensor, xmax: torch.Tensor,
                 rowptr_t: torch.Tensor, col_t: torch.Tensor, nbr_t: torch.Tensor,
                 ecount: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                                torch.Tensor, torch.Tensor]:
    """(dx, dW, dbias, dE1, dE2) of gcn_conv."""
    _cuda(g, x, W, rowptr_t, col_t, nbr_t, ecount)
    ctx = _Ctx(6)
    ctx.saved_tensors = (x.contiguous(), W)
    ctx.h3 = xmax.numel() > 0
    ctx.xmax = xmax
    ctx.params = (None, None, None, None)  # fresh gradient tensors
    ctx.graph = _graph_ns(None, col_t, None, rowptr_t, col_t, None, nbr_t, ecount)
    dx, dW, db, dE1, dE2, _ = ops._GCNConv.backward(ctx, g)
    return dx, dW, db, dE1, dE2


@gcn_conv_bwd.register_fake
def _(g, x, W, xmax, rowptr_t, col_t, nbr_t, ecount):
    return (torch.empty_like(x), torch.empty_like(W), W.new_empty(W.shape[1]), W.new_empty(5, 1),
            W.new_empty(3, 1))


# ---------------------------------------------------------------------------
# Linear -> ReLU -> Linear, and Linear
# ---------------------------------------------------------------------------
@custom_op("molclr::mlp", mutates_args=(), device_types="cuda")
def mlp(x: torch.Tensor, W1: torch.Tensor, b1: torch.Tensor, W2: torch.Tensor,
        b2: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """nn.Sequential(Linear, ReLU, Linear) (GINEConv.mlp, ginet_molclr.py:19-23,46-47;
    out_lin, :93-96) with the ReLU fused into the first product.  Returns (z,
    a1, bits, slots): a1 = relu(x W1^T + b1) and the backward's saved state
    (a1's ReLU bits and the h3 max slots; empty when the product is not h3)."""
    _cuda(x, W1, b1, W2, b2)
    if x.dim() != 2 or W1.shape != (b1.shape[0], x.shape[1]) or W2.shape != (b2.shape[0],
                                                                              W1.shape[0]):
        raise ValueError(f"mlp: shapes x {tuple(x.shape)}, W1 {tuple(W1.shape)}, b1 "
                         f"{tuple(b1.shape)}, W2 {tuple(W2.shape)}, b2 {tuple(b2.shape)}")
    ctx = _Ctx(6)
    z = ops._MLP.forward(ctx, x, W1, b1, W2, b2, False)
    a1 = ctx.saved_tensors[3]
    if ctx.h3:
        return z, a1, ctx.bits, ctx.slots
    return z, a1, x.new_empty(0, dtype=torch.int32), x.new_empty(0)


@mlp.register_fake
def _(x, W1, b1, W2, b2):
    M = x.shape[0]
    return (x.new_empty(M, W2.shape[0]), x.new_empty(M, W1.shape[0]),
            x.new_empty(0, dtype=torch.int32), x.new_empty(0))


@custom_op("molclr::mlp_bwd", mutates_args=(), device_types="cuda")
def mlp_bwd(dz: torch.Tensor, x: torch.Tensor, W1: torch.Tensor, W2: torch.Tensor,
            a1: torch.Tensor, bits: torch.Tensor, slots: torch.Tensor
            ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dx, dW1, db1, dW2, db2) of mlp."""
    _cuda(dz, x, W1, W2, a1)
    ctx = _Ctx(6)
    ctx.saved_tensors = (x.contiguous(), W1, W2, a1)
    ctx.params = (None, None, None, None)
    ctx.side = False
    ctx.h3 = bits.numel() > 0
    ctx.bits, ctx.slots = bits, slots
    dx, dW1, db1, dW2, db2, _ = ops._MLP.backward(ctx, dz)
    return dx, dW1, db1, dW2, db2


@mlp_bwd.register_fake
def _(dz, x, W1, W2, a1, bits, slots):
    return (torch.empty_like(x), torch.empty_like(W1), W1.new_empty(W1.shape[0]),
            torch.empty_like(W2), W2.new_empty(W2.shape[0]))


@custom_op("molclr::linear", mutates_args=(), device_types="cuda")
def linear(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """nn.Linear: x W^T + b (feat_lin, ginet_molclr.py:90-92,114), molclr_gemm_f32."""
    _cuda(x, W, b)
    if x.dim() != 2 or W.shape != (b.shape[0], x.shape[1]):
        raise ValueError(f"linear: x {tuple(x.shape)}, W {tuple(W.shape)}, b {tuple(b.shape)}")
    return ops._Linear.forward(_Ctx(4), x, W, b, False)


@linear.register_fake
def _(x, W, b):
    return x.new_empty(x.shape[0], W.shape[0])


@custom_op("molclr::linear_bwd", mutates_args=(), device_types="cuda")
def linear_bwd(dy: torch.Tensor, x: torch.Tensor, W: torch.Tensor
               ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dx, dW, db) of linear."""
    _cuda(dy, x, W)
    dx, dW, db = ops.linear_bwd(dy.contiguous(), x.contiguous(), W)
    return dx, dW, db


@linear_bwd.register_fake
def _(dy, x, W):
    return torch.empty_like(x), torch.empty_like(W), W.new_empty(W.shape[0])


# ---------------------------------------------------------------------------
# BatchNorm1d (+ ReLU) over row segments
# ---------------------------------------------------------------------------
def _seg_rows_arg(seg_rows, N):
    import ctypes
    rows = [int(r) for r in seg_rows]
    if not rows or any(r < 0 for r in rows) or sum(rows) != N:
        raise ValueError(f"batch_norm_seg: seg_rows {rows} must be >= 0 and sum to the {N} rows")
    return rows, (ctypes.c_int64 * len(rows))(*rows)


def _bn_dtype(z):
    if z.dtype == torch.float32:
        return _lib.DTYPE_F32
    if z.dtype == torch.bfloat16:
        return _lib.DTYPE_BF16
    raise TypeError(f"batch_norm_seg: {z.dtype} rows (fp32 / bf16)")


@custom_op("molclr::batch_norm_seg", mutates_args=(), device_types="cuda")
def batch_norm_seg(z: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                   running_mean: torch.Tensor | None, running_var: torch.Tensor | None,
                   num_batches_tracked: torch.Tensor | None, seg_rows: list[int],
                   training: bool, momentum: float, eps: float, relu: bool
                   ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor,
                              torch.Tensor, torch.Tensor]:
    """BatchNorm1d(D) (+ ReLU) over consecutive row segments, each normalised
    with its own batch statistics (training) -- the reference's one BatchNorm
    call per encoder call (ginet_molclr.py:105-111, two calls per step at
    molclr.py:57,60) -- with the running statistics updated once per segment
    in segment order (momentum, unbiased variance, num_batches_tracked += 1
    each), as torch.nn.BatchNorm1d would over the segments one by one.  Eval
    (training False): the running statistics, nothing updated.  Returns (y,
    save_mean [S, D], save_invstd [S, D], running_mean', running_var',
    num_batches_tracked'): the op is functional (autograd needs that), so the
    updated running statistics come back as new tensors (empty when not
    given); batch_norm_seg_module() writes them into an nn.BatchNorm1d."""
    _cuda(z, gamma, beta)
    z = z.contiguous()
    N, D = z.shape
    rows, c_rows = _seg_rows_arg(seg_rows, N)
    S = len(rows)
    for t in (running_mean, running_var):
        if t is not None and (tuple(t.shape) != (D,) or t.dtype != torch.float32 or not t.is_cuda):
            raise ValueError(f"batch_norm_seg: running statistics must be fp32 [{D}] on the GPU")
    if not training and (running_mean is None or running_var is None):
        raise ValueError("batch_norm_seg: eval mode needs the running statistics")
    dt = _bn_dtype(z)
    y = torch.empty_like(z)
    f32 = dict(dtype=torch.float32, device=z.device)
    mean, invstd = torch.empty(S, D, **f32), torch.empty(S, D, **f32)
    rm = running_mean.clone() if running_mean is not None else None
    rv = running_var.clone() if running_var is not None else None
    nbt = num_batches_tracked.clone() if num_batches_tracked is not None else None
    wsb = _lib.query("molclr_batchnorm_seg_workspace_bytes", S, c_rows, D)
    ws = ops._ws(wsb, z.device)
    _lib.call("molclr_batchnorm_seg_fwd", z.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
              _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(nbt), y.data_ptr(), mean.data_ptr(),
              invstd.data_ptr(), S, c_rows, D, dt, float(momentum), float(eps),
              int(bool(training)), int(bool(relu)), ws.data_ptr(), wsb, _stream(z))
    empty = z.new_empty(0, dtype=torch.float32)
    return (y, mean, invstd, rm if rm is not None else empty, rv if rv is not None else empty,
            nbt if nbt is not None else z.new_empty(0, dtype=torch.long))


def batch_norm_seg_module(z: torch.Tensor, bn: torch.nn.BatchNorm1d, seg_rows, relu: bool):
    """torch.ops.molclr.batch_norm_seg for an nn.BatchNorm1d (momentum set,
    affine), writing the updated running statistics back into ``bn`` in
    training mode; returns y."""
    if bn.momentum is None or not bn.affine:
        raise ValueError("batch_norm_seg_module: a BatchNorm1d with a momentum and affine weights")
    track = bn.track_running_stats
    training = bn.training or not track
    y, _, _, rm, rv, nbt = torch.ops.molclr.batch_norm_seg(
        z, bn.weight, bn.bias, bn.running_mean if track else None,
        bn.running_var if track else None, bn.num_batches_tracked if track else None,
        [int(r) for r in seg_rows], training, float(bn.momentum), float(bn.eps), bool(relu))
    if bn.training and track:
        with torch.no_grad():
            bn.running_mean.copy_(rm)
            bn.running_var.copy_(rv)
            bn.num_batches_tracked.copy_(nbt)
    return y


@batch_norm_seg.register_fake
def _(z, gamma, beta, running_mean, running_var, num_batches_tracked, seg_rows, training,
      momentum, eps, relu):
    S, D = len(seg_rows), z.shape[1]
    f32 = dict(dtype=torch.float32)
    return (torch.empty_like(z), z.new_empty(S, D, **f32), z.new_empty(S, D, **f32),
            z.new_empty(D if running_mean is not None else 0, **f32),
            z.new_empty(D if running_var is not None else 0, **f32),
            z.new_empty(() if num_batches_tracked is not None else (0,), dtype=torch.long))


@custom_op("molclr::batch_norm_seg_bwd", mutates_args=(), device_types="cuda")
def batch_norm_seg_bwd(dy: torch.Tensor, z: torch.Tensor, gamma: torch.Tensor,
                       beta: torch.Tensor, save_mean: torch.Tensor, save_invstd: torch.Tensor,
                       seg_rows: list[int], relu: bool
                       ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dz, dgamma, dbeta) of batch_norm_seg in training mode (dgamma / dbeta
    summed over the segments in segment order)."""
    _cuda(dy, z, gamma, beta, save_mean, save_invstd)
    z = z.contiguous()
    dy = dy.contiguous().to(z.dtype)
    N, D = z.shape
    rows, c_rows = _seg_rows_arg(seg_rows, N)
    S = len(rows)
    dt = _bn_dtype(z)
    dz = torch.empty_like(z)
    f32 = dict(dtype=torch.float32, device=z.device)
    dg, dbt = torch.empty(D, **f32), torch.empty(D, **f32)
    wsb = _lib.query("molclr_batchnorm_seg_workspace_bytes", S, c_rows, D)
    ws = ops._ws(wsb, z.device)
    _lib.call("molclr_batchnorm_seg_bwd", dy.data_ptr(), z.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), save_mean.data_ptr(), save_invstd.data_ptr(), dz.data_ptr(),
              dg.data_ptr(), dbt.data_ptr(), S, c_rows, D, dt, int(bool(relu)), 0, ws.data_ptr(),
              wsb, _stream(z))
    return dz, dg, dbt


@batch_norm_seg_bwd.register_fake
def _(dy, z, gamma, beta, save_mean, save_invstd, seg_rows, relu):
    D = z.shape[1]
    return torch.empty_like(z), gamma.new_empty(D), gamma.new_empty(D)

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


def _gcn_agg_setup(ctx, inputs, output):
    xw, E1, E2, bias, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount = inputs
    ctx.save_for_backward(rowptr_t, col_t, nbr_t, ecount)


def _gcn_agg_backward(ctx, g):
    dxw, dE1, dE2, db = torch.ops.molclr.gcn_aggregate_bwd(g, *ctx.saved_tensors)
    return (dxw, dE1, dE2, db) + (None,) * 8


gcn_aggregate.register_autograd(_gcn_agg_backward, setup_context=_gcn_agg_setup)


def _gcn_conv_setup(ctx, inputs, output):
    x, W, bias, E1, E2, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount = inputs
    ctx.save_for_backward(x, W, output[1], rowptr_t, col_t, nbr_t, ecount)


def _gcn_conv_backward(ctx, g, _gxmax):
    dx, dW, db, dE1, dE2 = torch.ops.molclr.gcn_conv_bwd(g, *ctx.saved_tensors)
    return (dx, dW, db, dE1, dE2) + (None,) * 8


gcn_conv.register_autograd(_gcn_conv_backward, setup_context=_gcn_conv_setup)


def _mlp_setup(ctx, inputs, output):
    x, W1, b1, W2, b2 = inputs
    z, a1, bits, slots = output
    ctx.save_for_backward(x, W1, W2, a1, bits, slots)


def _mlp_backward(ctx, dz, _ga1, _gbits, _gslots):
    x, W1, W2, a1, bits, slots = ctx.saved_tensors
    if _ga1 is not None and _ga1.abs().sum().item() != 0:
        raise RuntimeError("molclr::mlp: a1 is saved state, not a differentiable output")
    return torch.ops.molclr.mlp_bwd(dz, x, W1, W2, a1, bits, slots)


mlp.register_autograd(_mlp_backward, setup_context=_mlp_setup)


def _linear_setup(ctx, inputs, output):
    x, W, b = inputs
    ctx.save_for_backward(x, W)


def _linear_backward(ctx, dy):
    return torch.ops.molclr.linear_bwd(dy, *ctx.saved_tensors)


linear.register_autograd(_linear_backward, setup_context=_linear_setup)


def _bn_setup(ctx, inputs, output):
    z, gamma, beta, rm, rv, nbt, seg_rows, training, momentum, eps, relu = inputs
    y, mean, invstd = output[:3]
    ctx.save_for_backward(z, gamma, beta, mean, invstd)
    ctx.seg_rows, ctx.relu, ctx.training = list(seg_rows), bool(relu), bool(training)


def _bn_backward(ctx, dy, *_state):
    if not ctx.training:
        raise NotImplementedError("molclr::batch_norm_seg: no backward through eval mode (the "
                                  "reference evaluates under torch.no_grad, molclr.py:162)")
    z, gamma, beta, mean, invstd = ctx.saved_tensors
    dz, dg, db = torch.ops.molclr.batch_norm_seg_bwd(dy, z, gamma, beta, mean, invstd,
                                                     ctx.seg_rows, ctx.relu)
    return dz, dg, db, None, None, None, None, None, None, None, None


batch_norm_seg.register_autograd(_bn_backward, setup_context=_bn_setup)

OPS = ("graph_build", "gine_aggregate", "gine_aggregate_bwd", "segment_pool", "segment_pool_bwd",
       "l2_normalize", "l2_normalize_bwd", "nt_xent", "nt_xent_bwd", "gcn_aggregate",
       "gcn_aggregate_bwd", "gcn_conv", "gcn_conv_bwd", "mlp", "mlp_bwd", "linear", "linear_bwd",
       "batch_norm_seg", "batch_norm_seg_bwd")
