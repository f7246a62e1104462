"""dgl.nn.pytorch: SAGEConv (the reference's layer, code/model.py:7, 13-15) and GraphConv,
with DGL 0.8.2's constructor signatures, parameter names and initialisation, computed by
the plagnn engine."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import plagnn
from plagnn import ops


def _check_graph(graph):
    import dgl

    if not isinstance(graph, dgl.DGLGraph):
        raise TypeError("expected a dgl.DGLGraph built by this package")


class SAGEConv(nn.Module):
    """DGL 0.8.2 ``SAGEConv(in_feats, out_feats, aggregator_type, feat_drop=0., bias=True,
    norm=None, activation=None)``.

    'pool' (the reference's aggregator): ``relu(fc_pool(h))`` max-aggregated over in-edges,
    then ``fc_self(h) + fc_neigh(neigh) + bias``; the whole layer runs as one fused
    autograd function on the engine (ops.SagePool). 'mean' and 'gcn' are provided for
    the aggregator variants the reference does not use (reference-unpinned); 'lstm' is
    not supported.
    """

    def __init__(self, in_feats, out_feats, aggregator_type, feat_drop=0.0, bias=True,
                 norm=None, activation=None):
        super().__init__()
        valid = {"mean", "pool", "gcn", "lstm"}
        if aggregator_type not in valid:
            raise KeyError(f"Invalid aggregator_type. Must be one of {valid}. "
                           f"But got {aggregator_type!r} instead.")
        if aggregator_type == "lstm":
            raise NotImplementedError("SAGEConv 'lstm' is not provided by this engine")
        if isinstance(in_feats, tuple):
            if in_feats[0] != in_feats[1]:
                raise NotImplementedError("bipartite SAGEConv is not supported")
            in_feats = in_feats[0]
        self._in_src_feats = self._in_dst_feats = in_feats
        self._out_feats = out_feats
        self._aggre_type = aggregator_type
        self.norm = norm
        self.feat_drop = nn.Dropout(feat_drop)
        self.activation = activation
        if aggregator_type == "pool":
            self.fc_pool = nn.Linear(in_feats, in_feats)
        self.fc_neigh = nn.Linear(in_feats, out_feats, bias=False)
        if aggregator_type != "gcn":
            self.fc_self = nn.Linear(in_feats, out_feats, bias=False)
        if bias:
            self.bias = nn.parameter.Parameter(torch.zeros(out_feats))
        else:
            self.register_buffer("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        if self._aggre_type == "pool":
            nn.init.xavier_uniform_(self.fc_pool.weight, gain=gain)
        if self._aggre_type != "gcn":
            nn.init.xavier_uniform_(self.fc_self.weight, gain=gain)
        nn.init.xavier_uniform_(self.fc_neigh.weight, gain=gain)

    def forward(self, graph, feat, edge_weight=None):
        _check_graph(graph)
        if isinstance(feat, tuple):
            raise NotImplementedError("bipartite input features are not supported")
        feat = self.feat_drop(feat)
        dg = graph._device_graph(feat.device)
        ews = dg.edge_weight_slots(edge_weight)
        if self._aggre_type == "pool":
            rst = ops.SagePool.apply(feat.float(), self.fc_pool.weight, self.fc_pool.bias,
                                     self.fc_self.weight, self.fc_neigh.weight, self.bias, dg, ews)
        else:
            lin_before_mp = self._in_src_feats > self._out_feats
            h = self.fc_neigh(feat) if lin_before_mp else feat
            if self._aggre_type == "mean":
                h_neigh = ops.SumAggregate.apply(h, dg, ews, True)
            else:  # gcn: (sum of neighbours + self) / (in-degree + 1)
                s = ops.SumAggregate.apply(h, dg, ews, False)
                degs = torch.as_tensor(graph._engine_graph().in_degrees(), device=feat.device)
                h_neigh = (s + h) / (degs.unsqueeze(-1).to(feat.dtype) + 1)
            if not lin_before_mp:
                h_neigh = self.fc_neigh(h_neigh)
            rst = h_neigh if self._aggre_type == "gcn" else self.fc_self(feat) + h_neigh
            if self.bias is not None:
                rst = rst + self.bias
        if self.activation is not None:
            rst = self.activation(rst)
        if self.norm is not None:
            rst = self.norm(rst)
        return rst

    def extra_repr(self):
        return f"in={self._in_src_feats}, out={self._out_feats}, aggregator_type={self._aggre_type!r}"


class GraphConv(nn.Module):
    """DGL 0.8.2 ``GraphConv(in_feats, out_feats, norm='both', weight=True, bias=True,
    activation=None, allow_zero_in_degree=False)`` on the engine's sum aggregation.
    Not used by the reference (BASELINE config 0 names it): reference-unpinned."""

    def __init__(self, in_feats, out_feats, norm="both", weight=True, bias=True,
                 activation=None, allow_zero_in_degree=False):
        super().__init__()
        if norm not in ("none", "both", "right", "left"):
            raise ValueError(f'Invalid norm value. Must be either "none", "both", "right" or '
                             f'"left". But got "{norm}".')
        self._in_feats, self._out_feats, self._norm = in_feats, out_feats, norm
        self._allow_zero_in_degree = allow_zero_in_degree
        self.weight = nn.Parameter(torch.Tensor(in_feats, out_feats)) if weight else None
        self.bias = nn.Parameter(torch.Tensor(out_feats)) if bias else None
        self._activation = activation
        self.reset_parameters()

    def reset_parameters(self):
        if self.weight is not None:
            nn.init.xavier_uniform_(self.weight)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, graph, feat, weight=None, edge_weight=None):
        _check_graph(graph)
        dg = graph._device_graph(feat.device)
        eg = graph._engine_graph()
        if not self._allow_zero_in_degree and (eg.in_degrees() == 0).any():
            raise plagnn.PlagnnError("There are 0-in-degree nodes in the graph; add self-loops "
                                     "or set allow_zero_in_degree=True")
        ews = dg.edge_weight_slots(edge_weight)
        if self._norm in ("left", "both"):
            degs = torch.as_tensor(eg.out_degrees(), device=feat.device).float().clamp(min=1)
            norm = torch.pow(degs, -0.5) if self._norm == "both" else 1.0 / degs
            feat = feat * norm.reshape(-1, 1)
        w = weight if weight is not None else self.weight
        if self._in_feats > self._out_feats:
            if w is not None:
                feat = feat @ w
            rst = ops.SumAggregate.apply(feat, dg, ews, False)
        else:
            rst = ops.SumAggregate.apply(feat, dg, ews, False)
            if w is not None:
                rst = rst @ w
        if self._norm in ("right", "both"):
            degs = torch.as_tensor(eg.in_degrees(), device=feat.device).float().clamp(min=1)
            norm = torch.pow(degs, -0.5) if self._norm == "both" else 1.0 / degs
            rst = rst * norm.reshape(-1, 1)
        if self.bias is not None:
            rst = rst + self.bias
        if self._activation is not None:
            rst = self._activation(rst)
        return rst


__all__ = ["SAGEConv", "GraphConv"]
