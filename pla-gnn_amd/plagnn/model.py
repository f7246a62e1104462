"""GNN32 — the reference's model (code/model.py:10-31) on the engine's SAGEConv.

Same constructor, parameter names (conv{1,2,3}.fc_pool / fc_self / fc_neigh / bias,
liner1, liner2) and forward as the reference, so its state_dict and training loop carry
over unchanged. ``GNN`` generalises the depth (BASELINE configs: 2 or 3 SAGE layers)
while keeping the same naming scheme.
"""
from __future__ import annotations

from typing import Sequence

import torch as th
import torch.nn as nn
import torch.nn.functional as F

from dgl.nn.pytorch import GraphConv, SAGEConv


class GNN32(nn.Module):
    """code/model.py:10-31 (dropout argument accepted and unused, as there)."""

    def __init__(self, in_feats, h1_feats, h2_feats, h3_feats, h4_feats, num_classes,
                 dropout=0.5):
        super().__init__()
        self.conv1 = SAGEConv(in_feats, h1_feats, "pool")
        self.conv2 = SAGEConv(h1_feats, h2_feats, "pool")
        self.conv3 = SAGEConv(h2_feats, h3_feats, "pool")
        self.liner1 = nn.Linear(h3_feats, h4_feats)
        self.liner2 = nn.Linear(h4_feats, num_classes)

    def forward(self, g, in_feat):
        h = self.conv1(g, in_feat)
        h = F.leaky_relu(h)
        h = self.conv2(g, h)
        h = F.leaky_relu(h)
        h = self.conv3(g, h)
        h = F.leaky_relu(h)
        h = self.liner1(h)
        h = F.leaky_relu(h)
        h = self.liner2(h)
        return th.sigmoid(h)


class GNN(nn.Module):
    """GNN32 with any number of graph layers: dims = [in, h_1, ..., h_L, h_mlp, classes].
    conv = 'pool' (the reference's SAGEConv aggregator), or for BASELINE configs[0]
    ("2-layer GraphConv hidden=64"; not a configuration of the reference, reference-
    unpinned) 'graphconv' (dgl.nn.pytorch.GraphConv, norm 'both') and the SAGEConv
    variants 'mean' / 'gcn'."""

    def __init__(self, dims: Sequence[int], conv: str = "pool"):
        super().__init__()
        dims = list(dims)
        if len(dims) < 4:
            raise ValueError("dims = [in, h_1, ..., h_L, h_mlp, classes] with L >= 1")
        self.dims = dims
        self.conv = conv
        self.n_conv = len(dims) - 3
        for i in range(self.n_conv):
            if conv == "graphconv":
                layer = GraphConv(dims[i], dims[i + 1])
            elif conv in ("pool", "mean", "gcn"):
                layer = SAGEConv(dims[i], dims[i + 1], conv)
            else:
                raise ValueError(f"unknown conv {conv!r}")
            setattr(self, f"conv{i + 1}", layer)
        self.liner1 = nn.Linear(dims[-3], dims[-2])
        self.liner2 = nn.Linear(dims[-2], dims[-1])

    def forward(self, g, in_feat, edge_weight=None):
        h = in_feat
        for i in range(self.n_conv):
            h = F.leaky_relu(getattr(self, f"conv{i + 1}")(g, h, edge_weight=edge_weight))
        h = F.leaky_relu(self.liner1(h))
        return th.sigmoid(self.liner2(h))
