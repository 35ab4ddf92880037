"""Graph containers with the PyG 1.6.3 ``Data`` / ``Batch`` field contract.

The reference's encoders read ``data.x`` [N,2] int64 (atom type, chirality),
``data.edge_index`` [2,E] int64, ``data.edge_attr`` [E,2] int64 (bond type,
bond direction) and ``data.batch`` [N] int64 (models/ginet_molclr.py:99-101,113),
produced by dataset/dataset.py:86-147 and PyG's collate.  These classes keep
exactly that contract (so a real ``torch_geometric`` Batch can be passed
instead) and add :class:`DeviceGraph`, the once-per-batch CSR that replaces
PyG's per-layer ``add_self_loops`` + scatter bookkeeping.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Sequence

import torch

from . import _lib


class Data:
    """One molecule graph (torch_geometric.data.Data subset)."""

    def __init__(self, x=None, edge_index=None, edge_attr=None, **kwargs):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        return int(self.x.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.shape[1])

    def to(self, device, non_blocking: bool = False):
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            if k.startswith("_molclr"):
                continue
            out.__dict__[k] = v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v
        return out

    def __repr__(self) -> str:
        fields = ", ".join(f"{k}={list(v.shape)}" for k, v in self.__dict__.items()
                           if torch.is_tensor(v))
        return f"{self.__class__.__name__}({fields})"


class Batch(Data):
    """A disjoint union of graphs (torch_geometric.data.Batch subset)."""

    @staticmethod
    def from_data_list(data_list: Sequence[Data]) -> "Batch":
        """PyG 1.6.3 collate: concatenate x/edge_attr, offset edge_index by the
        running node count, build the ascending ``batch`` vector and ``ptr``."""
        xs, eis, eas, bs = [], [], [], []
        offset = 0
        ptr = [0]
        for g, d in enumerate(data_list):
            n = d.num_nodes
            xs.append(d.x)
            eis.append(d.edge_index + offset)
            eas.append(d.edge_attr)
            bs.append(torch.full((n,), g, dtype=torch.long))
            offset += n
            ptr.append(offset)
        b = Batch(
            x=torch.cat(xs, 0),
            edge_index=torch.cat(eis, 1),
            edge_attr=torch.cat(eas, 0),
            batch=torch.cat(bs, 0),
        )
        b.ptr = torch.tensor(ptr, dtype=torch.long)
        b._num_graphs = len(data_list)
        return b

    @property
    def num_graphs(self) -> int:
        if getattr(self, "_num_graphs", None) is not None:
            return self._num_graphs
        if getattr(self, "ptr", None) is not None:
            return int(self.ptr.numel() - 1)
        return int(self.batch.max().item()) + 1 if self.batch.numel() else 0

    def to(self, device, non_blocking: bool = False):
        out = super().to(device, non_blocking)
        out._num_graphs = self.num_graphs
        return out


def collate_pairs(pairs: Iterable[tuple]) -> tuple:
    """Collate a list of (view_i, view_j) molecule pairs into (Batch_i, Batch_j),
    as the reference DataLoader does for MoleculeDataset (dataset.py:147,179)."""
    pairs = list(pairs)
    return (Batch.from_data_list([p[0] for p in pairs]),
            Batch.from_data_list([p[1] for p in pairs]))


def _num_graphs_of(data) -> int:
    ng = getattr(data, "num_graphs", None)
    if ng is not None:
        return int(ng)
    b = getattr(data, "batch", None)
    if b is None:
        return 1
    return int(b.max().item()) + 1 if b.numel() else 0


class DeviceGraph:
    """Destination CSR / source CSC / bond-type counts / graph offsets of one
    batch, built on the GPU by ``molclr_graph_build`` (graph.hip).

    :meth:`union` builds the graph of several batches taken as one
    (``molclr_graph_build_multi``): the two contrastive views of a step run
    through one encoder pass, ``segment_nodes`` telling the executors where
    each view's rows start (their BatchNorm statistics stay per view)."""

    def __init__(self, edge_index: torch.Tensor, edge_attr: torch.Tensor, num_nodes: int,
                 batch: torch.Tensor | None = None, num_graphs: int | None = None):
        dev = edge_index.device
        if batch is None:
            batch = torch.zeros(int(num_nodes), dtype=torch.long, device=dev)
            num_graphs = 1 if int(num_nodes) > 0 else 0
        self._build([(edge_index, edge_attr, batch, int(num_nodes), int(num_graphs))])

    @classmethod
    def union(cls, parts) -> "DeviceGraph":
        """parts: (edge_index, edge_attr, batch, num_nodes, num_graphs) per batch."""
        g = cls.__new__(cls)
        g._build(list(parts))
        return g

    def _build(self, parts):
        dev = parts[0][0].device
        if dev.type != "cuda":
            raise RuntimeError("DeviceGraph: molclr_amd runs on the GPU only (got %s)" % dev)
        if not 1 <= len(parts) <= _lib.MAX_SEGMENTS:
            raise ValueError(f"DeviceGraph: {len(parts)} segments (1..{_lib.MAX_SEGMENTS})")
        keep = []  # the int64 inputs must outlive the (asynchronous) build
        segs = (_lib.GraphSegmentC * len(parts))()
        for q, (ei, ea, b, n, G) in enumerate(parts):
            ei = ei.to(torch.long).contiguous()
            ea = ea.to(torch.long).contiguous()
            b = b.to(torch.long).contiguous()
            keep += [ei, ea, b]
            segs[q] = _lib.GraphSegmentC(ei.data_ptr(), ea.data_ptr(), b.data_ptr(), int(n),
                                         int(ei.shape[1]), int(G))
        N = sum(int(p[3]) for p in parts)
        E = sum(int(segs[q].num_edges) for q in range(len(parts)))
        G = sum(int(p[4]) for p in parts)
        i32 = dict(dtype=torch.int32, device=dev)
        self.num_nodes, self.num_edges, self.num_graphs = N, E, G
        self.segment_nodes = [int(p[3]) for p in parts]
        self.rowptr = torch.empty(N + 1, **i32)
        self.col = torch.empty(max(E, 1), **i32)
        self.ecode = torch.empty(max(E, 1), dtype=torch.uint8, device=dev)
        self.rowptr_t = torch.empty(N + 1, **i32)
        self.col_t = torch.empty(max(E, 1), **i32)
        self.nbr = torch.empty(max(N, 1) * 4, **i32)    # neighbour slots (molclr.h)
        self.nbr_t = torch.empty(max(N, 1) * 4, **i32)
        self.ecount = torch.empty(max(N, 1) * 8, **i32)
        self.graph_ptr = torch.empty(G + 1, **i32)
        self.status = torch.empty(1, **i32)
        ws_bytes = _lib.query("molclr_graph_build_workspace_bytes", N, E)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _lib.call("molclr_graph_build_multi", len(parts), ctypes.addressof(segs),
                  self.rowptr.data_ptr(), self.col.data_ptr(), self.ecode.data_ptr(),
                  self.rowptr_t.data_ptr(), self.col_t.data_ptr(), self.nbr.data_ptr(),
                  self.nbr_t.data_ptr(), self.ecount.data_ptr(), self.graph_ptr.data_ptr(),
                  self.status.data_ptr(), ws.data_ptr(), ws_bytes, _lib.stream_of(dev))
        self.device = dev

    def cstruct(self):
        """struct molclr_device_graph of this graph (for the encoder executor)."""
        c = getattr(self, "_cstruct", None)
        if c is None:
            c = _lib.DeviceGraphC(self.num_nodes, self.num_edges, self.num_graphs, *[
                t.data_ptr() for t in (self.rowptr, self.col, self.rowptr_t, self.col_t,
                                       self.ecount, self.graph_ptr, self.ecode, self.nbr,
                                       self.nbr_t)])
            c.num_segments = len(self.segment_nodes)
            for q, n in enumerate(self.segment_nodes):
                c.segment_nodes[q] = n
            self._cstruct = c
        return c

    def check(self) -> None:
        """Synchronising validity check of the input indices (tests / debug)."""
        raise_for_status(int(self.status.item()))


def raise_for_status(st: int) -> None:
    """ValueError naming every invalid-input bit of a graph status word."""
    if st:
        what = []
        if st & 1:
            what.append("edge_index out of range")
        if st & 2:
            what.append("edge_attr out of range")
        if st & 4:
            what.append("batch not ascending / out of range")
        if st & _lib.STATUS_ATOM_RANGE:
            what.append("atom type / chirality outside the model's embedding tables "
                        "(the reference's nn.Embedding raises IndexError)")
        raise ValueError("invalid graph batch: " + ", ".join(what))


def pair_graph(xi, xj) -> DeviceGraph:
    """The graph of both views of a step as one (view i first), cached on xi."""
    g = getattr(xi, "_molclr_pair_graph", None)
    if g is not None and g[0] is xj and g[1].device == xi.edge_index.device:
        return g[1]
    parts = []
    for d in (xi, xj):
        b = getattr(d, "batch", None)
        n = int(d.x.shape[0])
        if b is None:
            b = torch.zeros(n, dtype=torch.long, device=d.edge_index.device)
        parts.append((d.edge_index, d.edge_attr, b, n, _num_graphs_of(d)))
    g = DeviceGraph.union(parts)
    try:
        xi._molclr_pair_graph = (xj, g)
    except AttributeError:
        pass
    return g


def device_graph(data) -> DeviceGraph:
    """The DeviceGraph of a Batch, built once and cached on the object."""
    g = getattr(data, "_molclr_graph", None)
    if g is not None and g.device == data.edge_index.device:
        return g
    g = DeviceGraph(data.edge_index, data.edge_attr, data.x.shape[0],
                    getattr(data, "batch", None), _num_graphs_of(data))
    try:
        data._molclr_graph = g
    except AttributeError:
        pass
    return g
