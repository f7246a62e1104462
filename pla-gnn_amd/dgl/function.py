"""dgl.function builtins understood by DGLGraph.update_all (the forms SAGEConv uses:
copy_u('h', 'm') / u_mul_e('h', '_edge_weight', 'm') with sum / mean / max)."""
from __future__ import annotations


class _Message:
    def __init__(self, op: str, lhs: str, rhs, out: str):
        self.op, self.lhs, self.rhs, self.out = op, lhs, rhs, out


class _Reduce:
    def __init__(self, op: str, msg: str, out: str):
        self.op, self.msg, self.out = op, msg, out


def copy_u(u: str, out: str) -> _Message:
    return _Message("copy_u", u, None, out)


copy_src = copy_u  # DGL < 0.8 name


def u_mul_e(lhs_field: str, rhs_field: str, out: str) -> _Message:
    return _Message("u_mul_e", lhs_field, rhs_field, out)


def sum(msg: str, out: str) -> _Reduce:  # noqa: A001  (DGL's name)
    return _Reduce("sum", msg, out)


def mean(msg: str, out: str) -> _Reduce:
    return _Reduce("mean", msg, out)


def max(msg: str, out: str) -> _Reduce:  # noqa: A001  (DGL's name)
    return _Reduce("max", msg, out)
