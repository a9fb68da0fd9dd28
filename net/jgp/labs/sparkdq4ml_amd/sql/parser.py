"""Recursive-descent parser for the Spark SQL subset the lab uses:

    SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0
    SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0

(``DataQuality4MachineLearningApp.java:77-78,89-90``) — projections with ``CAST``, aliases with or
without ``AS``, single-table ``FROM`` of a temp view, ``WHERE`` with arithmetic / comparisons /
boolean logic / ``IS [NOT] NULL`` / ``BETWEEN`` / ``IN``, ``CASE WHEN``, ``LIMIT``, UDF and
built-in function calls.  It produces the same plan nodes as the DataFrame API.
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

from .expressions import (Alias, AnalysisException, BinOp, CaseWhen, Cast, ColRef, Coalesce,
                          Expr, If, IsNotNull, IsNull, Lit, Neg, Not, UdfCall)
from .fn import MathFn, BUILTIN_MATH
from .plan import Filter, Limit, Project

__all__ = ["parse_expression", "parse_select_item", "plan_sql", "ParseException"]


class ParseException(AnalysisException):
    pass


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[dDlL]?)
  | (?P<str>'(?:[^'\\]|\\.|'')*')
  | (?P<bq>`[^`]+`)
  | (?P<ident>[A-Za-z_][A-Za-z_0-9]*)
  | (?P<op><=>|<=|>=|<>|!=|==|\|\||[=<>+\-*/%(),.])
""", re.VERBOSE)

_KEYWORDS = {"select", "from", "where", "as", "and", "or", "not", "cast", "is", "null", "true", "false",
             "case", "when", "then", "else", "end", "limit", "between", "in", "distinct", "like"}


def _tokenize(text: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ParseException(f"\nmismatched input '{text[pos]}' expecting <EOF>(line 1, pos {pos})")
        pos = m.end()
        kind = m.lastgroup
        val = m.group(kind)
        if kind == "ws":
            continue
        if kind == "ident" and val.lower() in _KEYWORDS:
            out.append(("kw", val.lower()))
        elif kind == "bq":
            out.append(("ident", val[1:-1]))
        else:
            out.append((kind, val))
    out.append(("eof", ""))
    return out


class _Parser:
    def __init__(self, text):
        self.toks = _tokenize(text)
        self.i = 0
        self.text = text

    def peek(self, k=0):
        return self.toks[self.i + k]

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, val=None):
        t = self.peek()
        if t[0] == kind and (val is None or t[1].lower() == val):
            self.i += 1
            return t
        return None

    def expect(self, kind, val=None):
        t = self.accept(kind, val)
        if t is None:
            got = self.peek()
            raise ParseException(f"\nmismatched input '{got[1] or '<EOF>'}' expecting {val or kind}")
        return t

    # ---- query -------------------------------------------------------------------------------
    def query(self, session):
        return _bind_query(self.query_syntax(), self.text, session)

    def query_syntax(self):
        """The statement's syntax: (select items, view name, alias, WHERE, LIMIT) -- nothing of
        the catalog is read here, so the result is cached per text (``plan_sql``)."""
        self.expect("kw", "select")
        self.accept("kw", "distinct")
        items = self.select_list()
        self.expect("kw", "from")
        tname = self.expect("ident")[1]
        alias = None
        if self.accept("kw", "as"):
            alias = self.expect("ident")[1]
        elif self.peek()[0] == "ident":
            alias = self.next()[1]
        where = None
        if self.accept("kw", "where"):
            where = self.expr()
        limit = None
        if self.accept("kw", "limit"):
            limit = int(self.expect("num")[1])
        self.expect("eof")
        quals = {tname.lower()} | ({alias.lower()} if alias else set())
        items = [(_strip_qual(e, quals)) for e in items]
        if where is not None:
            where = _strip_qual(where, quals)
        return items, tname, where, limit

    def select_list(self):
        items = [self.select_item()]
        while self.accept("op", ","):
            items.append(self.select_item())
        return items

    def select_item(self):
        if self.accept("op", "*"):
            return ColRef("*")
        e = self.expr()
        if self.accept("kw", "as"):
            return Alias(e, self.expect("ident")[1])
        if self.peek()[0] == "ident":
            return Alias(e, self.next()[1])
        return e

    # ---- expressions ---------------------------------------------------------------------------
    def expr(self):
        return self.or_()

    def or_(self):
        e = self.and_()
        while self.accept("kw", "or"):
            e = BinOp("or", e, self.and_())
        return e

    def and_(self):
        e = self.not_()
        while self.accept("kw", "and"):
            e = BinOp("and", e, self.not_())
        return e

    def not_(self):
        if self.accept("kw", "not"):
            return Not(self.not_())
        return self.predicate()

    def predicate(self):
        e = self.additive()
        t = self.peek()
        if t[0] == "op" and t[1] in ("=", "==", "<", ">", "<=", ">=", "<>", "!=", "<=>"):
            self.next()
            return BinOp(t[1], e, self.additive())
        if self.accept("kw", "is"):
            neg = bool(self.accept("kw", "not"))
            self.expect("kw", "null")
            return IsNotNull(e) if neg else IsNull(e)
        neg = bool(self.accept("kw", "not"))
        if self.accept("kw", "between"):
            lo = self.additive()
            self.expect("kw", "and")
            hi = self.additive()
            r = BinOp("and", BinOp(">=", e, lo), BinOp("<=", e, hi))
            return Not(r) if neg else r
        if self.accept("kw", "in"):
            self.expect("op", "(")
            vals = [self.expr()]
            while self.accept("op", ","):
                vals.append(self.expr())
            self.expect("op", ")")
            r = BinOp("=", e, vals[0])
            for v in vals[1:]:
                r = BinOp("or", r, BinOp("=", e, v))
            return Not(r) if neg else r
        if neg:
            raise ParseException("\nmismatched input 'NOT'")
        return e

    def additive(self):
        e = self.mult()
        while self.peek()[0] == "op" and self.peek()[1] in ("+", "-"):
            op = self.next()[1]
            e = BinOp(op, e, self.mult())
        return e

    def mult(self):
        e = self.unary()
        while self.peek()[0] == "op" and self.peek()[1] in ("*", "/", "%"):
            op = self.next()[1]
            e = BinOp(op, e, self.unary())
        return e

    def unary(self):
        if self.accept("op", "-"):
            e = self.unary()
            if isinstance(e, Lit) and isinstance(e.value, (int, float)) and not isinstance(e.value, bool):
                return Lit(-e.value, e.dtype)
            return Neg(e)
        if self.accept("op", "+"):
            return self.unary()
        return self.primary()

    def primary(self):
        t = self.next()
        kind, val = t
        if kind == "num":
            v = val.lower()
            if v.endswith("d"):
                return Lit(float(v[:-1]))
            if v.endswith("l"):
                from .types import LongType

                return Lit(int(v[:-1]), LongType())
            if "." in v or "e" in v:
                return Lit(float(v))
            return Lit(int(v))
        if kind == "str":
            return Lit(val[1:-1].replace("''", "'").replace("\\'", "'"))
        if kind == "kw":
            if val == "null":
                return Lit(None)
            if val in ("true", "false"):
                return Lit(val == "true")
            if val == "cast":
                self.expect("op", "(")
                e = self.expr()
                self.expect("kw", "as")
                tname = self.expect("ident")[1]
                if self.accept("op", "("):
                    args = [self.expect("num")[1]]
                    while self.accept("op", ","):
                        args.append(self.expect("num")[1])
                    self.expect("op", ")")
                    tname += "(" + ",".join(args) + ")"
                self.expect("op", ")")
                return Cast(e, tname)
            if val == "case":
                branches = []
                operand = None
                if not (self.peek()[0] == "kw" and self.peek()[1] == "when"):
                    operand = self.expr()
                while self.accept("kw", "when"):
                    c = self.expr()
                    if operand is not None:
                        c = BinOp("=", operand, c)
                    self.expect("kw", "then")
                    branches.append((c, self.expr()))
                other = None
                if self.accept("kw", "else"):
                    other = self.expr()
                self.expect("kw", "end")
                return CaseWhen(branches, other)
            raise ParseException(f"\nmismatched input '{val}'")
        if kind == "op" and val == "(":
            e = self.expr()
            self.expect("op", ")")
            return e
        if kind == "ident":
            if self.accept("op", "("):
                args = []
                if not self.accept("op", ")"):
                    args.append(self.expr())
                    while self.accept("op", ","):
                        args.append(self.expr())
                    self.expect("op", ")")
                return _function(val, args)
            if self.accept("op", "."):
                field = self.expect("ident")[1]
                return ColRef(val + "." + field)
            return ColRef(val)
        raise ParseException(f"\nmismatched input '{val or '<EOF>'}'")


def _function(name: str, args: List[Expr]) -> Expr:
    low = name.lower()
    if low == "coalesce":
        return Coalesce(*args)
    if low == "isnull":
        return IsNull(args[0])
    if low == "isnotnull":
        return IsNotNull(args[0])
    if low == "if":
        return If(*args)
    if low in BUILTIN_MATH:
        return MathFn(low, args)
    return UdfCall(name, args)


def _strip_qual(e: Expr, quals) -> Expr:
    """``p.guest`` -> ``guest`` when ``p`` names the FROM relation."""
    if isinstance(e, ColRef) and "." in e.name:
        q, _, f = e.name.partition(".")
        if q.lower() in quals:
            return ColRef(f)
        return e
    for attr in ("child", "left", "right", "cond", "a", "b", "otherwise"):
        if hasattr(e, attr) and isinstance(getattr(e, attr), Expr):
            setattr(e, attr, _strip_qual(getattr(e, attr), quals))
    if hasattr(e, "args"):
        e.args = [_strip_qual(a, quals) for a in e.args]
    if hasattr(e, "branches"):
        e.branches = [(_strip_qual(c, quals), _strip_qual(v, quals)) for c, v in e.branches]
    return e


def parse_expression(text: str) -> Expr:
    p = _Parser(text)
    e = p.expr()
    p.expect("eof")
    return e


def parse_select_item(text: str) -> Expr:
    p = _Parser(text)
    e = p.select_item()
    p.expect("eof")
    return e


_BOUND: dict = {}  # (statement, view plan skey) -> analyzed [Filter?, Project, Limit?] templates


def _bind_query(syntax, text: str, session):
    """The plan of a parsed SELECT over the session's CURRENT view of its FROM name (a temp view
    replaced between two runs of the same text binds to the new plan).  Expression trees are
    immutable once parsed, so plans may share them; a statement bound over a view of the same
    structure (sql/skey.py) reuses the analyzed nodes (fresh copies: no result is shared)."""
    items, tname, where, limit = syntax
    plan = session.catalog._views.get(tname.lower())
    if plan is None:
        raise AnalysisException(f"Table or view not found: {tname}; line 1 pos {text.lower().find(tname.lower())}")
    vk = plan.skey()
    key = (text, vk) if vk is not None else None
    tmpl = _BOUND.get(key) if key is not None else None
    if tmpl is not None:
        for t in tmpl:
            plan = t.fresh(plan)
        return plan
    out = _bind_new(items, where, limit, plan)
    if key is not None and out.skey() is not None:
        nodes, p = [], out
        while p is not plan:
            nodes.append(p)
            p = p.child
        tmpl = []
        for n in reversed(nodes):  # bottom-up, detached from the lineage
            n.schema()
            t = n.fresh()
            t.child = None
            tmpl.append(t)
        if len(_BOUND) >= 1024:
            _BOUND.clear()
        _BOUND[key] = tmpl
    return out


def _bind_new(items, where, limit, plan):
    if where is not None:
        plan = Filter(plan, where)
    exprs = []
    for e in items:
        if isinstance(e, ColRef) and e.name == "*":
            exprs += [ColRef(n) for n in plan.schema().names]
        else:
            exprs.append(e)
    plan = Project(plan, exprs)
    cs = plan.child.schema()
    for e in exprs:
        e.data_type(cs)
    if limit is not None:
        plan = Limit(plan, limit)
    return plan


_SYNTAX: dict = {}


def plan_sql(text: str, session):
    """``spark.sql(text)``: Spark re-parses every statement; the app re-runs the same two
    statements on every action (``DataQuality4MachineLearningApp.java:77-78, 89-90``), so the
    syntax is parsed once per text and only bound to the current catalog per call."""
    syn = _SYNTAX.get(text)
    if syn is None:
        syn = _Parser(text).query_syntax()
        if len(_SYNTAX) >= 256:
            _SYNTAX.clear()
        _SYNTAX[text] = syn
    return _bind_query(syn, text, session)


_ = Optional
