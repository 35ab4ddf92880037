"""GIN-E encoder + projection head — drop-in for models/ginet_molclr.py.

Same class names, constructor arguments, parameter-creation order (hence the
same seeded initialisation) and ``state_dict`` keys as the reference
(models/ginet_molclr.py:16-117): ``x_embedding{1,2}.weight``,
``gnns.{l}.mlp.{0,2}.{weight,bias}``, ``gnns.{l}.edge_embedding{1,2}.weight``,
``batch_norms.{l}.*``, ``feat_lin.*``, ``out_lin.{0,2}.*``.  The forward runs
entirely on the HIP kernels of libmolclr_hip.so (see molclr_amd.ops).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import ops
from .data import DeviceGraph, device_graph, pair_graph

num_atom_type = 119  # including the extra mask tokens
num_chirality_tag = 3

num_bond_type = 5  # including aromatic and self-loop edge
num_bond_direction = 3


class GINEConv(nn.Module):
    """GIN-E convolution, models/ginet_molclr.py:16-47.

    ``out_i = MLP( Σ_{j→i} (x_j + e_ji) + (x_i + e_self) )`` with
    ``e = E1[bond type] + E2[bond dir]`` and the self loop (type 4, dir 0).
    """

    def __init__(self, emb_dim):
        super().__init__()
        self.mlp = nn.Sequential(
            nn.Linear(emb_dim, 2 * emb_dim),
            nn.ReLU(),
            nn.Linear(2 * emb_dim, emb_dim),
        )
        self.edge_embedding1 = nn.Embedding(num_bond_type, emb_dim)
        self.edge_embedding2 = nn.Embedding(num_bond_direction, emb_dim)
        nn.init.xavier_uniform_(self.edge_embedding1.weight.data)
        nn.init.xavier_uniform_(self.edge_embedding2.weight.data)

    def aggregate(self, x, graph: DeviceGraph, Ec=None):
        """Ec: this layer's combined edge table (ops.edge_tables_combine), or None."""
        return ops.gine_aggregate(x, self.edge_embedding1.weight, self.edge_embedding2.weight,
                                  graph, Ec)

    def update(self, aggr_out):
        return ops.gin_mlp(aggr_out, self.mlp[0].weight, self.mlp[0].bias, self.mlp[2].weight,
                           self.mlp[2].bias)

    def forward(self, x, edge_index, edge_attr, graph: DeviceGraph | None = None):
        if graph is None:
            graph = DeviceGraph(edge_index, edge_attr, x.shape[0])
        return self.update(self.aggregate(x, graph))


class GINet(nn.Module):
    """models/ginet_molclr.py:50-117.  ``forward(data) -> (h [B, feat_dim],
    out [B, feat_dim // 2])``."""

    def __init__(self, num_layer=5, emb_dim=300, feat_dim=256, drop_ratio=0, pool='mean',
                 precision='fp32'):
        super().__init__()
        if precision not in ('fp32', 'bf16'):
            raise ValueError(f"precision {precision!r}: 'fp32' or 'bf16'")
        # 'bf16': the c5 configuration (BASELINE.json) / the reference's
        # fp16_precision switch (molclr.py:16-24,93-96): bf16 node features and
        # bf16 MFMA GEMMs with fp32 accumulation; fp32 master weights, BatchNorm
        # statistics, pooled features, heads and NT-Xent
        self.precision = precision
        self.num_layer = num_layer
        self.emb_dim = emb_dim
        self.feat_dim = feat_dim
        self.drop_ratio = drop_ratio

        self.x_embedding1 = nn.Embedding(num_atom_type, emb_dim)
        self.x_embedding2 = nn.Embedding(num_chirality_tag, emb_dim)
        nn.init.xavier_uniform_(self.x_embedding1.weight.data)
        nn.init.xavier_uniform_(self.x_embedding2.weight.data)

        self.gnns = nn.ModuleList()
        for _ in range(num_layer):
            self.gnns.append(GINEConv(emb_dim))

        self.batch_norms = nn.ModuleList()
        for _ in range(num_layer):
            self.batch_norms.append(nn.BatchNorm1d(emb_dim))

        # The reference leaves self.pool unset for an unknown name and fails at
        # forward time (ginet_molclr.py:83-88); fail at construction instead.
        if pool not in ('mean', 'add', 'max'):
            raise ValueError('Not defined pooling!')
        self.pool = pool

        self.feat_lin = nn.Linear(self.emb_dim, self.feat_dim)

        self.out_lin = nn.Sequential(
            nn.Linear(self.feat_dim, self.feat_dim),
            nn.ReLU(inplace=True),
            nn.Linear(self.feat_dim, self.feat_dim // 2),
        )

    # Run the node-embedding stack through the native encoder executor
    # (ops.gin_encoder, one host call per direction) when its BatchNorm and
    # dropout settings are the ones it implements; else op by op.
    use_executor = True

    def _executor_ok(self) -> bool:
        # any emb_dim: the executor runs on the width padded to the kernels'
        # multiple (_dim_pad) with zero columns
        if not self.use_executor or self.num_layer > 16:
            return False
        if self.drop_ratio > 0 and self.training:
            return False
        bn0 = self.batch_norms[0]
        return all(bn.track_running_stats and bn.affine and bn.momentum is not None
                   and bn.training == bn0.training and bn.momentum == bn0.momentum
                   and bn.eps == bn0.eps for bn in self.batch_norms)

    def _dim_pad(self) -> int:
        """Zero columns that bring emb_dim to the kernels' multiple (4 fp32, 8 bf16)."""
        return (-self.emb_dim) % (8 if self.precision == 'bf16' else 4)

    def _encoder_params(self):
        params = [self.x_embedding1.weight, self.x_embedding2.weight]
        for g, bn in zip(self.gnns, self.batch_norms):
            params += [g.mlp[0].weight, g.mlp[0].bias, g.mlp[2].weight, g.mlp[2].bias,
                       g.edge_embedding1.weight, g.edge_embedding2.weight, bn.weight, bn.bias]
        p = self._dim_pad()
        if not p:
            return params
        # emb_dim D -> D + p (hidden 2D -> 2D + 2p) with zero rows / columns
        # (F.pad: the gradients of the real entries flow back, the pads' drop).
        # A zero column stays zero through every layer: embeddings and edge
        # tables add 0, the Linear weights' zero rows / columns keep it out of
        # the real columns, and BatchNorm with gamma = beta = 0 maps it to 0.
        out = [F.pad(params[0], (0, p)), F.pad(params[1], (0, p))]
        for l in range(self.num_layer):
            W0, b0, W2, b2, E1, E2, g, b = params[2 + 8 * l: 2 + 8 * (l + 1)]
            out += [F.pad(W0, (0, p, 0, 2 * p)), F.pad(b0, (0, 2 * p)),
                    F.pad(W2, (0, 2 * p, 0, p)), F.pad(b2, (0, p)),
                    F.pad(E1, (0, p)), F.pad(E2, (0, p)), F.pad(g, (0, p)), F.pad(b, (0, p))]
        return out

    def _run_encoder(self, x, graph):
        """ops.gin_encoder on the (padded) width; returns h [N, emb_dim + pad]."""
        p = self._dim_pad()
        bns = list(self.batch_norms)
        if p:  # running statistics on the padded width, copied back after the call
            bns = [_PaddedBatchNorm(bn, p) for bn in bns]
        h = ops.gin_encoder(x, graph, bns, self._encoder_params(), self.precision)
        if p:
            for pb in bns:
                pb.copy_back()
        return h

    def encode(self, data, graph: DeviceGraph | None = None):
        """Node embeddings after the last layer (ginet_molclr.py:103-111)."""
        graph = graph or device_graph(data)
        if self._executor_ok():
            h = self._run_encoder(data.x, graph)
            return (h[:, :self.emb_dim] if self._dim_pad() else h), graph
        if self.precision != 'fp32':
            raise NotImplementedError("bf16 runs through the encoder executor only "
                                      "(dropout 0, tracked BatchNorm statistics)")
        if self._dim_pad():
            raise NotImplementedError("emb_dim %% 4 != 0 runs through the encoder executor only "
                                      "(dropout 0, tracked BatchNorm statistics)")
        h = ops.atom_embed(data.x, self.x_embedding1.weight, self.x_embedding2.weight,
                           graph.status)
        # per-edge embeddings E1[bt] + E2[bd] of every layer, tabulated in one launch
        Ec = ops.edge_tables_combine([g.edge_embedding1.weight for g in self.gnns],
                                     [g.edge_embedding2.weight for g in self.gnns])
        for layer in range(self.num_layer):
            h = self.gnns[layer].update(self.gnns[layer].aggregate(h, graph, Ec[layer]))
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
        """Both contrastive views of a step in ONE pass: ``(h, out)`` with the
        rows of ``forward(xi)`` followed by those of ``forward(xj)``
        (molclr.py:57,60).  The views' graphs are built as one
        (molclr_graph_build_multi) and every BatchNorm keeps per-view batch
        statistics, updating its running statistics for view i, then view j
        (molclr_batchnorm_seg_fwd) -- the two-call semantics, with half the
        launches and twice the rows per GEMM / aggregation launch."""
        if not self._executor_ok():
            hi, oi = self(xi)
            hj, oj = self(xj)
            return torch.cat([hi, hj], 0), torch.cat([oi, oj], 0)
        graph = pair_graph(xi, xj)
        x = torch.cat([xi.x, xj.x], 0)
        return self._readout(self._run_encoder(x, graph), graph)


class _PaddedBatchNorm:
    """A BatchNorm1d's settings and running statistics on the padded width
    (GINet._run_encoder); copy_back() writes the real columns back."""

    def __init__(self, bn: nn.BatchNorm1d, p: int):
        self.bn = bn
        self.training, self.momentum, self.eps = bn.training, bn.momentum, bn.eps
        self.num_batches_tracked = bn.num_batches_tracked
        self.running_mean = F.pad(bn.running_mean, (0, p))
        self.running_var = F.pad(bn.running_var, (0, p), value=1.0)

    def copy_back(self):
        D = self.bn.running_mean.shape[0]
        self.bn.running_mean.copy_(self.running_mean[:D])
        self.bn.running_var.copy_(self.running_var[:D])
