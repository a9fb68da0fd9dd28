"""Structural keys of expressions and logical plans: the host-issue side of an action
(SURVEY.md §3 'Catalyst analysis per action').

Spark re-analyzes every action's freshly built DataFrame (``DataQuality4MachineLearningApp.java:53-126``
runs the whole chain again for each ``fit``).  Here the analysis results are shared by structure: a
plan node's key is an interned integer built from its operator, its expressions and its child's
key, so two actions that build the same chain over the same input get the same keys, and

* the analyzed schema of a Project (``plan.Project.schema``),
* a DataFrame transformation's analyzed plan node (``dataframe.DataFrame._derive``: the result is a
  fresh node copied from the first one, with the caller's child, so no execution result is ever
  shared between actions),
* the lowered fused-scan fit of an action (``models.regression``),

are computed once per structure.  Keys are exact: every expression field takes part (UDFs by the
registry entry they resolve to, literals by type and value, data types by their SQL name), and a
field the walk cannot key (an array, an arbitrary object) makes the whole expression unkeyable
(``None``: no sharing)."""
from __future__ import annotations

from typing import Optional

__all__ = ["intern", "expr_key", "pin", "clear"]

_INTERN: dict = {}
_PINNED: dict = {}  # identity-keyed objects, kept alive so that an id is never reused in a key


def intern(t) -> int:
    k = _INTERN.get(t)
    if k is None:
        if len(_INTERN) >= 1 << 20:  # unbounded structure churn: start over (keys stay unique per epoch)
            clear()
        k = _INTERN[t] = len(_INTERN) + 1 + _EPOCH[0]
    return k


_EPOCH = [0]


def clear() -> None:
    _EPOCH[0] += 1 << 21
    _INTERN.clear()
    _PINNED.clear()


def pin(obj) -> tuple:
    """An identity key for ``obj`` (a registered UDF, a cached file entry) that stays unique: the
    object is kept alive for as long as keys may mention it."""
    _PINNED[id(obj)] = obj
    return ("id", id(obj))


class _Unkeyable(Exception):
    pass


_T = {}  # lazily bound classes (sql.expressions imports this module's users, not the reverse)


def _classes():
    if not _T:
        from .expressions import ColRef, Expr, UdfCall
        from .types import DataType

        _T.update(Expr=Expr, DataType=DataType, ColRef=ColRef, UdfCall=UdfCall)
    return _T


def _val(v):
    T = _T or _classes()
    Expr, DataType = T["Expr"], T["DataType"]
    if isinstance(v, Expr):
        k = expr_key(v)
        if k is None:
            raise _Unkeyable
        return k
    if v is None or isinstance(v, (bool, int, str)):
        return (type(v).__name__, v)
    if isinstance(v, float):
        return ("float", repr(v))
    if isinstance(v, (list, tuple)):
        return ("seq",) + tuple(_val(x) for x in v)
    if isinstance(v, DataType):
        return ("dt", type(v).__name__, v.simpleString())
    raise _Unkeyable


def expr_key(e) -> Optional[int]:
    """Interned structural key of an expression tree (cached on the node), or None."""
    d = e.__dict__
    if "_skey" in d:
        return d["_skey"]
    T = _T or _classes()
    try:
        if type(e) is T["ColRef"]:  # (the common leaf: one small tuple)
            k = d["_skey"] = intern(("col", e.name))
            return k
        if isinstance(e, T["UdfCall"]):
            u = e._resolved()
            t = ("UdfCall", e.name, pin(u)) + tuple(_val(a) for a in e.args)
        else:
            t = (type(e).__module__, type(e).__qualname__) + tuple(
                (n, _val(v)) for n, v in d.items() if not n.startswith("_"))
        k = intern(t)
    except _Unkeyable:
        k = None
    except Exception:  # an unresolvable UDF etc.: analysis reports it, keys just opt out
        k = None
    d["_skey"] = k
    return k


def exprs_key(exprs) -> Optional[tuple]:
    ks = tuple(expr_key(e) for e in exprs)
    return None if None in ks else ks
