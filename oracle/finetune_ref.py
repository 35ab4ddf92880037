"""ORACLE — test infrastructure only (see oracle/__init__.py).

The parameter layout of the reference's fine-tuning models
(models/ginet_finetune.py:52-127, GINet(task, num_layer, emb_dim, feat_dim,
drop_ratio, pool, pred_n_layer, pred_act); models/gcn_finetune.py:94-157,
GCN(task, num_layer, emb_dim, feat_dim, drop_ratio, pool)) and their
checkpoint loader ``load_my_state_dict`` (ginet_finetune.py:149-157,
gcn_finetune.py:166-174, called from finetune.py:247-257), restated
to check that a pre-training checkpoint written by molclr_amd fits it: the
module tree and names are what a state_dict exposes, so only the
constructor's layout is restated (the forward is not needed for the check).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from oracle.reference_cpu import (num_atom_type, num_bond_direction, num_bond_type,
                                  num_chirality_tag)


class _GINEConvLayout(nn.Module):
    def __init__(self, emb_dim):  # ginet_finetune.py:16-28
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(emb_dim, 2 * emb_dim), nn.ReLU(),
                                 nn.Linear(2 * emb_dim, emb_dim))
        self.edge_embedding1 = nn.Embedding(num_bond_type, emb_dim)
        self.edge_embedding2 = nn.Embedding(num_bond_direction, emb_dim)


class FinetuneGINetLayout(nn.Module):
    """ginet_finetune.py:62-127: encoder as in pre-training, feat_lin, and the
    task head pred_head (no out_lin)."""

    def __init__(self, task="classification", num_layer=5, emb_dim=300, feat_dim=512,
                 pred_n_layer=2, pred_act="softplus"):
        super().__init__()
        self.x_embedding1 = nn.Embedding(num_atom_type, emb_dim)
        self.x_embedding2 = nn.Embedding(num_chirality_tag, emb_dim)
        self.gnns = nn.ModuleList([_GINEConvLayout(emb_dim) for _ in range(num_layer)])
        self.batch_norms = nn.ModuleList([nn.BatchNorm1d(emb_dim) for _ in range(num_layer)])
        self.feat_lin = nn.Linear(emb_dim, feat_dim)
        out_dim = 2 if task == "classification" else 1
        act = {"relu": lambda: nn.ReLU(inplace=True), "softplus": nn.Softplus}[pred_act]
        head = [nn.Linear(feat_dim, feat_dim // 2), act()]
        for _ in range(max(1, pred_n_layer) - 1):
            head += [nn.Linear(feat_dim // 2, feat_dim // 2), act()]
        head.append(nn.Linear(feat_dim // 2, out_dim))
        self.pred_head = nn.Sequential(*head)

    def load_my_state_dict(self, state_dict):
        """ginet_finetune.py:149-157: copy every entry whose name the model
        has (a shape mismatch raises in copy_), skip the rest."""
        own = self.state_dict()
        for name, param in state_dict.items():
            if name not in own:
                continue
            if isinstance(param, nn.parameter.Parameter):
                param = param.data
            own[name].copy_(param)


class _GCNConvLayout(nn.Module):
    def __init__(self, emb_dim):  # gcn_finetune.py:39-53
        super().__init__()
        self.weight = nn.Parameter(torch.empty(emb_dim, emb_dim))
        self.bias = nn.Parameter(torch.empty(emb_dim))
        self.edge_embedding1 = nn.Embedding(num_bond_type, 1)
        self.edge_embedding2 = nn.Embedding(num_bond_direction, 1)


class FinetuneGCNLayout(nn.Module):
    """gcn_finetune.py:94-141: the pre-training GCN encoder, feat_lin, and the
    task head pred_lin = Linear(feat, feat/2), Softplus, Linear(feat/2, 2 | 1)
    (no out_lin)."""

    def __init__(self, task="classification", num_layer=5, emb_dim=300, feat_dim=256):
        super().__init__()
        if num_layer < 2:
            raise ValueError("Number of GNN layers must be greater than 1.")
        self.x_embedding1 = nn.Embedding(num_atom_type, emb_dim)
        self.x_embedding2 = nn.Embedding(num_chirality_tag, emb_dim)
        self.gnns = nn.ModuleList([_GCNConvLayout(emb_dim) for _ in range(num_layer)])
        self.batch_norms = nn.ModuleList([nn.BatchNorm1d(emb_dim) for _ in range(num_layer)])
        self.feat_lin = nn.Linear(emb_dim, feat_dim)
        out_dim = 2 if task == "classification" else 1
        self.pred_lin = nn.Sequential(nn.Linear(feat_dim, feat_dim // 2), nn.Softplus(),
                                      nn.Linear(feat_dim // 2, out_dim))

    load_my_state_dict = FinetuneGINetLayout.load_my_state_dict
