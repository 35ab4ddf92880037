"""GCN encoder + projection head — drop-in for models/gcn_molclr.py.

Same names, constructor arguments, parameter-creation order and state_dict
keys as the reference (models/gcn_molclr.py:39-158; keys verified against the
shipped ``ckpt/pretrained_gcn/checkpoints/model.pth``):
``gnns.{l}.{weight,bias,edge_embedding1.weight,edge_embedding2.weight}``.

The reference computes ``gcn_norm`` and discards the result
(gcn_molclr.py:74), so it has no effect on outputs and is not computed; the
``torch_sparse`` ``message_and_aggregate`` path (gcn_molclr.py:90-91) is dead
for dense ``edge_index`` input and is not provided.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import Parameter

from . import ops
from .ginet_molclr import _PaddedBatchNorm
from .data import DeviceGraph, device_graph, pair_graph

num_atom_type = 119  # including the extra mask tokens
num_chirality_tag = 3

num_bond_type = 5  # including aromatic and self-loop edge
num_bond_direction = 3


class GCNConv(nn.Module):
    """models/gcn_molclr.py:39-91:
    ``out_i = Σ_{j→i} (e_ji + (xW)_j) + (e_self + (xW)_i) + b``, scalar e."""

    def __init__(self, emb_dim, aggr="add"):
        super().__init__()
        if aggr != "add":
            raise NotImplementedError("molclr_amd GCNConv supports aggr='add' (the reference's)")
        self.emb_dim = emb_dim
        self.aggr = aggr

        self.weight = Parameter(torch.Tensor(emb_dim, emb_dim))
        self.bias = Parameter(torch.Tensor(emb_dim))
        self.reset_parameters()

        self.edge_embedding1 = nn.Embedding(num_bond_type, 1)
        self.edge_embedding2 = nn.Embedding(num_bond_direction, 1)

        nn.init.xavier_uniform_(self.edge_embedding1.weight.data)
        nn.init.xavier_uniform_(self.edge_embedding2.weight.data)

    def reset_parameters(self):
        stdv = math.sqrt(6.0 / (self.weight.size(-2) + self.weight.size(-1)))
        self.weight.data.uniform_(-stdv, stdv)
        self.bias.data.fill_(0)

    def conv(self, x, graph: DeviceGraph):
        return ops.gcn_conv(x, self.weight, self.bias, self.edge_embedding1.weight,
                            self.edge_embedding2.weight, graph)

    def forward(self, x, edge_index, edge_attr, graph: DeviceGraph | None = None):
        if graph is None:
            graph = DeviceGraph(edge_index, edge_attr, x.shape[0])
        return self.conv(x, graph)


class GCN(nn.Module):
    """models/gcn_molclr.py:94-158."""

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

        self.gnns = nn.ModuleList()
        for _ in range(num_layer):
            self.gnns.append(GCNConv(emb_dim, aggr="add"))

        self.batch_norms = nn.ModuleList()
        for _ in range(num_layer):
            self.batch_norms.append(nn.BatchNorm1d(emb_dim))

        if pool in ('mean', 'add', 'max'):
            self.pool = pool
        else:
            raise ValueError('Not defined pooling!')

        self.feat_lin = nn.Linear(self.emb_dim, self.feat_dim)

        self.out_lin = nn.Sequential(
            nn.Linear(self.feat_dim, self.feat_dim),
            nn.ReLU(inplace=True),
            nn.Linear(self.feat_dim, self.feat_dim // 2),
        )

    # Run the node-embedding stack through the native encoder executor
    # (ops.gcn_encoder, one host call per direction) when its BatchNorm and
    # dropout settings are the ones it implements; else op by op.
    use_executor = True

    def _executor_ok(self) -> bool:
        # any emb_dim: the executor runs on the width padded to a multiple of 4
        if not self.use_executor or self.num_layer > 16:
            return False
        if self.drop_ratio > 0 and self.training:
            return False
        bn0 = self.batch_norms[0]
        return all(bn.track_running_stats and bn.affine and bn.momentum is not None
                   and bn.training == bn0.training and bn.momentum == bn0.momentum
                   and bn.eps == bn0.eps for bn in self.batch_norms)

    def _dim_pad(self) -> int:
        return (-self.emb_dim) % 4

    def _encoder_params(self):
        params = [self.x_embedding1.weight, self.x_embedding2.weight]
        for g, bn in zip(self.gnns, self.batch_norms):
            params += [g.weight, g.bias, g.edge_embedding1.weight, g.edge_embedding2.weight,
                       bn.weight, bn.bias]
        p = self._dim_pad()
        if not p:
            return params
        # zero-padded width (GINet._encoder_params); the scalar edge terms reach
        # the pad columns, and BatchNorm's zero gamma / beta map them back to 0
        out = [F.pad(params[0], (0, p)), F.pad(params[1], (0, p))]
        for l in range(self.num_layer):
            W, b, E1, E2, g, bb = params[2 + 6 * l: 2 + 6 * (l + 1)]
            out += [F.pad(W, (0, p, 0, p)), F.pad(b, (0, p)), E1, E2, F.pad(g, (0, p)),
                    F.pad(bb, (0, p))]
        return out

    def _run_encoder(self, x, graph):
        p = self._dim_pad()
        bns = list(self.batch_norms)
        if p:
            bns = [_PaddedBatchNorm(bn, p) for bn in bns]
        h = ops.gcn_encoder(x, graph, bns, self._encoder_params())
        if p:
            for pb in bns:
                pb.copy_back()
        return h

    def encode(self, data, graph: DeviceGraph | None = None):
        graph = graph or device_graph(data)
        if self._executor_ok():
            h = self._run_encoder(data.x, graph)
            return (h[:, :self.emb_dim] if self._dim_pad() else h), graph
        if self._dim_pad():
            raise NotImplementedError("emb_dim % 4 != 0 runs through the encoder executor only "
                                      "(dropout 0, tracked BatchNorm statistics)")
        h = ops.atom_embed(data.x, self.x_embedding1.weight, self.x_embedding2.weight,
                           graph.status)
        for layer in range(self.num_layer):
            h = self.gnns[layer].conv(h, graph)
            last = layer == self.num_layer - 1
            h = ops.batch_norm(h, self.batch_norms[layer], relu=not last)
            if self.drop_ratio > 0 and self.training:
                h = F.dropout(h, self.drop_ratio, training=True)
        return h, graph

    def _readout(self, h, graph):
        h = ops.segment_pool(h, graph, self.pool)
        W = self.feat_lin.weight
        if h.shape[1] != W.shape[1]:  # padded width: zero weight columns for the pads
            W = F.pad(W, (0, h.shape[1] - W.shape[1]))
        h = ops.linear(h, W, self.feat_lin.bias, side=True)
        out = ops.projection_head(h, self.out_lin[0].weight, self.out_lin[0].bias,
                                  self.out_lin[2].weight, self.out_lin[2].bias, side=True)
        return h, out

    def forward(self, data):
        if self._executor_ok():  # keep the padded width into the readout
            graph = device_graph(data)
            return self._readout(self._run_encoder(data.x, graph), graph)
        h, graph = self.encode(data)
        return self._readout(h, graph)

    def forward_staged(self, graph):
        """forward_pair over a StagedPairGraph (molclr_amd.graph_step): the
        views' atoms are graph.x, fixed-capacity buffers whose padding rows
        carry no gradient -- the capturable form of the paired pass."""
        if not self._executor_ok() or self._dim_pad():
            raise NotImplementedError("forward_staged needs the encoder executor at a width "
                                      "the kernels take unpadded")
        return self._readout(self._run_encoder(graph.x, graph), graph)

    def forward_pair(self, xi, xj):
        """Both views in one pass, per-view BatchNorm statistics (see
        GINet.forward_pair): rows of forward(xi) then forward(xj)."""
        if not self._executor_ok():
            hi, oi = self(xi)
            hj, oj = self(xj)
            return torch.cat([hi, hj], 0), torch.cat([oi, oj], 0)
        graph = pair_graph(xi, xj)
        x = torch.cat([xi.x, xj.x], 0)
        return self._readout(self._run_encoder(x, graph), graph)
