"""ORACLE — test infrastructure only (see oracle/__init__.py).

A line-by-line CPU restatement (torch, fp32) of the reference pre-training
step, with the absent third-party pieces restated from their published
behaviour:

* ``torch-geometric==1.6.3`` (README.md:37-38; not importable here, not
  vendored): ``add_self_loops`` appends ``[arange N; arange N]`` AFTER the
  real edges; ``MessagePassing.propagate`` with ``aggr='add'`` and
  ``flow='source_to_target'`` gathers ``x_j = x.index_select(0, edge_index[0])``,
  calls ``message``, scatter-adds at ``edge_index[1]`` with
  ``dim_size = N``, then ``update``; ``global_mean_pool`` = scatter-mean by
  ``batch`` (sum / count.clamp(1), size = batch.max() + 1).
* ``torch-scatter==2.0.6``: ``scatter_sum`` = ``zeros(...).scatter_add_``
  (CPU: accumulates in index order).

Module structure, parameter-creation order and state_dict keys follow
models/ginet_molclr.py:16-117 and models/gcn_molclr.py:27-158 so that the same
``torch.manual_seed`` gives the same weights as the reference would.
``RefNTXentLoss`` restates utils/nt_xent.py:5-65 including the broadcast
CosineSimilarity that materialises a (2B, 2B, C) tensor — that is the
reference's CPU cost, which the bench's ``cpu_baseline`` leg measures.

``RefGINet(..., emulate_bf16=True)`` is the same model with the HIP bf16
path's storage points (the c5 configuration, include/molclr.h "bf16
storage"): node features, aggregation outputs, MLP activations, BatchNorm
inputs and outputs and their gradients are rounded to bf16 where the kernels
store them, and the MLP weights enter their products as bf16; everything in
between stays in the oracle's precision (the kernels accumulate in fp32).

Parity status: the NT-Xent restatement is pinned by golden vectors produced
by importing the reference's own utils/nt_xent.py (tests/golden/).  The
encoder restatement cannot be pinned by reference outputs (the reference
encoders import torch_geometric, which is absent and stays absent): it is
checked against known-answer cases derived by hand from the reference
semantics and against the shipped pretrained_gcn checkpoint's key/shape
manifest — "parity partially unpinned" (DESIGN.md).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import Parameter

num_atom_type = 119  # models/ginet_molclr.py:9-13
num_chirality_tag = 3
num_bond_type = 5
num_bond_direction = 3


# ---------------------------------------------------------------------------
# PyG 1.6.3 / torch_scatter 2.0.6 semantics
# ---------------------------------------------------------------------------
def add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """torch_geometric.utils.add_self_loops: loops appended after the edges."""
    loop = torch.arange(num_nodes, dtype=torch.long, device=edge_index.device)
    loop = loop.unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index, loop], dim=1)


def scatter_sum(src: torch.Tensor, index: torch.Tensor, dim_size: int) -> torch.Tensor:
    """torch_scatter.scatter_sum along dim 0."""
    size = list(src.shape)
    size[0] = dim_size
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return torch.zeros(size, dtype=src.dtype).scatter_add_(0, idx, src)


def propagate_add(x_src: torch.Tensor, edge_index: torch.Tensor, num_nodes: int, message):
    """MessagePassing.propagate(aggr='add', flow='source_to_target')."""
    x_j = x_src.index_select(0, edge_index[0])
    msg = message(x_j)
    return scatter_sum(msg, edge_index[1], num_nodes)


def global_mean_pool(h: torch.Tensor, batch: torch.Tensor, size: int | None = None):
    size = int(batch.max().item()) + 1 if size is None else size
    s = scatter_sum(h, batch, size)
    cnt = scatter_sum(torch.ones(h.shape[0], dtype=h.dtype), batch, size).clamp(min=1)
    return s / cnt.unsqueeze(-1)


def global_add_pool(h: torch.Tensor, batch: torch.Tensor, size: int | None = None):
    size = int(batch.max().item()) + 1 if size is None else size
    return scatter_sum(h, batch, size)


def global_max_pool(h: torch.Tensor, batch: torch.Tensor, size: int | None = None):
    """PyG 1.6.3 global_max_pool = torch_scatter 2.0.6 scatter(reduce='max')
    (scatter_max): per graph and column the maximum; a graph without nodes
    pools to 0; the gradient goes to the arg-max node, the first in node order
    among equal values (torch_scatter's CPU loop keeps a strictly greater
    value; torch.max(dim) returns the first maximal index and routes its
    gradient there)."""
    size = int(batch.max().item()) + 1 if size is None else size
    rows = []
    for g in range(size):
        seg = h[batch == g]
        rows.append(seg.max(dim=0).values if seg.shape[0] else h.new_zeros(h.shape[1]))
    return torch.stack(rows)


# ---------------------------------------------------------------------------
# bf16 storage points of the HIP c5 path (emulate_bf16)
# ---------------------------------------------------------------------------
def _to_bf16(t: torch.Tensor) -> torch.Tensor:
    """Round to the nearest bf16 (even on ties), via fp32 as the kernels do."""
    return t.float().to(torch.bfloat16).to(t.dtype)


class _StoreBF16(torch.autograd.Function):
    """A tensor the kernels store in bf16: the value rounded in the forward,
    its gradient (also stored in bf16 by the backward kernels) in the backward."""

    @staticmethod
    def forward(ctx, x):
        return _to_bf16(x)

    @staticmethod
    def backward(ctx, g):
        return _to_bf16(g)


class _OperandBF16(torch.autograd.Function):
    """A weight used as a bf16 GEMM operand (the fp32 master is rounded; its
    gradient is fp32)."""

    @staticmethod
    def forward(ctx, w):
        return _to_bf16(w)

    @staticmethod
    def backward(ctx, g):
        return g


def _identity(t):
    return t


# ---------------------------------------------------------------------------
# models/ginet_molclr.py
# ---------------------------------------------------------------------------
class RefGINEConv(nn.Module):
    def __init__(self, emb_dim):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(emb_dim, 2 * emb_dim), nn.ReLU(),
                                 nn.Linear(2 * emb_dim, emb_dim))
        self.edge_embedding1 = nn.Embedding(num_bond_type, emb_dim)
        self.edge_embedding2 = nn.Embedding(num_bond_direction, emb_dim)
        nn.init.xavier_uniform_(self.edge_embedding1.weight.data)
        nn.init.xavier_uniform_(self.edge_embedding2.weight.data)

    def forward(self, x, edge_index, edge_attr):                     # ginet_molclr.py:29-41
        N = x.size(0)
        edge_index = add_self_loops(edge_index, N)
        self_loop_attr = torch.zeros(N, 2)
        self_loop_attr[:, 0] = 4
        self_loop_attr = self_loop_attr.to(edge_attr.device).to(edge_attr.dtype)
        edge_attr = torch.cat((edge_attr, self_loop_attr), dim=0)
        edge_embeddings = self.edge_embedding1(edge_attr[:, 0]) + self.edge_embedding2(edge_attr[:, 1])
        aggr = propagate_add(x, edge_index, N, lambda x_j: x_j + edge_embeddings)  # :43-44
        if not getattr(self, "emulate_bf16", False):
            return self.mlp(aggr)                                      # :46-47
        st, op = _StoreBF16.apply, _OperandBF16.apply
        lin1, lin2 = self.mlp[0], self.mlp[2]
        a1 = st(F.relu(F.linear(st(aggr), op(lin1.weight), lin1.bias)))
        return st(F.linear(a1, op(lin2.weight), lin2.bias))


class RefGINet(nn.Module):
    def __init__(self, num_layer=5, emb_dim=300, feat_dim=256, drop_ratio=0, pool='mean',
                 emulate_bf16=False):
        super().__init__()
        self.emulate_bf16 = emulate_bf16
        self.num_layer = num_layer
        self.emb_dim = emb_dim
        self.feat_dim = feat_dim
        self.drop_ratio = drop_ratio
        self.x_embedding1 = nn.Embedding(num_atom_type, emb_dim)
        self.x_embedding2 = nn.Embedding(num_chirality_tag, emb_dim)
        nn.init.xavier_uniform_(self.x_embedding1.weight.data)
        nn.init.xavier_uniform_(self.x_embedding2.weight.data)
        self.gnns = nn.ModuleList([RefGINEConv(emb_dim) for _ in range(num_layer)])
        for g in self.gnns:
            g.emulate_bf16 = emulate_bf16
        self.batch_norms = nn.ModuleList([nn.BatchNorm1d(emb_dim) for _ in range(num_layer)])
        self.pool = {'mean': global_mean_pool, 'add': global_add_pool,
                     'max': global_max_pool}[pool]                      # ginet_molclr.py:83-88
        self.feat_lin = nn.Linear(self.emb_dim, self.feat_dim)
        self.out_lin = nn.Sequential(nn.Linear(self.feat_dim, self.feat_dim), nn.ReLU(inplace=True),
                                     nn.Linear(self.feat_dim, self.feat_dim // 2))

    def forward(self, data):                                          # ginet_molclr.py:98-117
        st = _StoreBF16.apply if getattr(self, "emulate_bf16", False) else _identity
        x, edge_index, edge_attr = data.x, data.edge_index, data.edge_attr
        h = st(self.x_embedding1(x[:, 0]) + self.x_embedding2(x[:, 1]))
        for layer in range(self.num_layer):
            h = self.gnns[layer](h, edge_index, edge_attr)
            h = self.batch_norms[layer](h)
            if layer == self.num_layer - 1:
                h = F.dropout(h, self.drop_ratio, training=self.training)
            else:
                h = F.dropout(F.relu(h), self.drop_ratio, training=self.training)
            h = st(h)
        h = self.pool(h, data.batch)
        h = self.feat_lin(h)
        out = self.out_lin(h)
        return h, out


# ---------------------------------------------------------------------------
# models/gcn_molclr.py
# ---------------------------------------------------------------------------
class RefGCNConv(nn.Module):
    def __init__(self, emb_dim, aggr="add"):
        super().__init__()
        self.emb_dim = emb_dim
        self.aggr = aggr
        self.weight = Parameter(torch.Tensor(emb_dim, emb_dim))
        self.bias = Parameter(torch.Tensor(emb_dim))
        stdv = math.sqrt(6.0 / (self.weight.size(-2) + self.weight.size(-1)))  # :55-60
        self.weight.data.uniform_(-stdv, stdv)
        self.bias.data.fill_(0)
        self.edge_embedding1 = nn.Embedding(num_bond_type, 1)
        self.edge_embedding2 = nn.Embedding(num_bond_direction, 1)
        nn.init.xavier_uniform_(self.edge_embedding1.weight.data)
        nn.init.xavier_uniform_(self.edge_embedding2.weight.data)

    def forward(self, x, edge_index, edge_attr):                     # gcn_molclr.py:62-84
        N = x.size(0)
        edge_index = add_self_loops(edge_index, N)
        self_loop_attr = torch.zeros(N, 2)
        self_loop_attr[:, 0] = 4
        self_loop_attr = self_loop_attr.to(edge_attr.device).to(edge_attr.dtype)
        edge_attr = torch.cat((edge_attr, self_loop_attr), dim=0)
        edge_embeddings = self.edge_embedding1(edge_attr[:, 0]) + self.edge_embedding2(edge_attr[:, 1])
        # gcn_norm(edge_index) at :74 — its result is discarded by the reference
        x = x @ self.weight
        out = propagate_add(x, edge_index, N, lambda x_j: edge_embeddings + x_j)  # :86-88
        out = out + self.bias
        return out


class RefGCN(nn.Module):
    def __init__(self, num_layer=5, emb_dim=300, feat_dim=256, drop_ratio=0, pool='mean'):
        super().__init__()
        self.num_layer = num_layer
        self.emb_dim = emb_dim
        self.feat_dim = feat_dim
        self.drop_ratio = drop_ratio
        if self.num_layer < 2:
            raise ValueError("Number of GNN layers must be greater than 1.")
        self.x_embedding1 = nn.Embedding(num_atom_type, emb_dim)
        self.x_embedding2 = nn.Embedding(num_chirality_tag, emb_dim)
        nn.init.xavier_uniform_(self.x_embedding1.weight.data)
        nn.init.xavier_uniform_(self.x_embedding2.weight.data)
        self.gnns = nn.ModuleList([RefGCNConv(emb_dim, aggr="add") for _ in range(num_layer)])
        self.batch_norms = nn.ModuleList([nn.BatchNorm1d(emb_dim) for _ in range(num_layer)])
        self.pool = {'mean': global_mean_pool, 'add': global_add_pool,
                     'max': global_max_pool}[pool]                      # gcn_molclr.py:121-128
        self.feat_lin = nn.Linear(self.emb_dim, self.feat_dim)
        self.out_lin = nn.Sequential(nn.Linear(self.feat_dim, self.feat_dim), nn.ReLU(inplace=True),
                                     nn.Linear(self.feat_dim, self.feat_dim // 2))

    forward = RefGINet.forward


# ---------------------------------------------------------------------------
# utils/nt_xent.py
# ---------------------------------------------------------------------------
class RefNTXentLoss(nn.Module):
    def __init__(self, device, batch_size, temperature, use_cosine_similarity):
        super().__init__()
        self.batch_size = batch_size
        self.temperature = temperature
        self.device = device
        self.mask_samples_from_same_repr = self._get_correlated_mask().type(torch.bool)
        self.use_cosine = use_cosine_similarity
        self._cosine_similarity = nn.CosineSimilarity(dim=-1)
        self.criterion = nn.CrossEntropyLoss(reduction="sum")

    def _get_correlated_mask(self):                                  # nt_xent.py:24-30
        diag = np.eye(2 * self.batch_size)
        l1 = np.eye((2 * self.batch_size), 2 * self.batch_size, k=-self.batch_size)
        l2 = np.eye((2 * self.batch_size), 2 * self.batch_size, k=self.batch_size)
        mask = torch.from_numpy((diag + l1 + l2))
        mask = (1 - mask).type(torch.bool)
        return mask.to(self.device)

    def similarity(self, x, y):                                      # nt_xent.py:33-45
        if self.use_cosine:
            return self._cosine_similarity(x.unsqueeze(1), y.unsqueeze(0))
        return torch.tensordot(x.unsqueeze(1), y.T.unsqueeze(0), dims=2)

    def forward(self, zis, zjs):                                     # nt_xent.py:47-65
        representations = torch.cat([zjs, zis], dim=0)
        similarity_matrix = self.similarity(representations, representations)
        l_pos = torch.diag(similarity_matrix, self.batch_size)
        r_pos = torch.diag(similarity_matrix, -self.batch_size)
        positives = torch.cat([l_pos, r_pos]).view(2 * self.batch_size, 1)
        negatives = similarity_matrix[self.mask_samples_from_same_repr].view(2 * self.batch_size, -1)
        logits = torch.cat((positives, negatives), dim=1)
        logits /= self.temperature
        labels = torch.zeros(2 * self.batch_size).to(self.device).long()
        loss = self.criterion(logits, labels)
        return loss / (2 * self.batch_size)


# ---------------------------------------------------------------------------
# molclr.py: the step
# ---------------------------------------------------------------------------
def ref_step_loss(model, criterion, xis, xjs):
    """MolCLR._step (molclr.py:55-67)."""
    ris, zis = model(xis)
    rjs, zjs = model(xjs)
    zis = F.normalize(zis, dim=1)
    zjs = F.normalize(zjs, dim=1)
    return criterion(zis, zjs)


def ref_train_step(model, criterion, optimizer, xis, xjs):
    """One iteration of the hot loop (molclr.py:108-128)."""
    optimizer.zero_grad()
    loss = ref_step_loss(model, criterion, xis, xjs)
    loss.backward()
    optimizer.step()
    return loss.detach()
