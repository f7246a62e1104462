"""dgl.nn — PyTorch backend only (the reference uses dgl.nn.pytorch, code/model.py:7)."""
from . import pytorch  # noqa: F401
from .pytorch import GraphConv, SAGEConv  # noqa: F401
