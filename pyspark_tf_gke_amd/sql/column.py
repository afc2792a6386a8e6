"""Column expressions (``pyspark.sql.Column`` surface) and their compilation.

An expression tree is compiled per DataFrame batch into the register bytecode of the device
expression VM (csrc/kernels/df.hip ``expr_eval_k``): one fused pass over the rows evaluates the
whole tree — the role Catalyst's whole-stage codegen plays for the reference's filters and
``withColumn(when(...).otherwise(...))`` imputation (k_means.py:23-51).  CPU batches evaluate the
same tree with torch host ops (identical null semantics: SQL three-valued logic, division by zero
-> null, isnan(null) = false).
"""
from __future__ import annotations

import math

import torch

from . import types as T

BIN = {"+": "ADD", "-": "SUB", "*": "MUL", "/": "DIV", "%": "MOD", "==": "EQ", "!=": "NE", "<": "LT", "<=": "LE",
       ">": "GT", ">=": "GE", "&": "AND", "|": "OR", "pow": "POW", "<=>": "EQ_NULLSAFE", "least": "MIN2",
       "greatest": "MAX2", "coalesce": "COALESCE"}
CMP = {"EQ", "NE", "LT", "LE", "GT", "GE", "EQ_NULLSAFE"}
BOOL_OUT = CMP | {"AND", "OR", "NOT", "ISNULL", "ISNOTNULL", "ISNAN"}


def _wrap(x) -> "Column":
    if isinstance(x, Column):
        return x
    return Column(("lit", x))


class Column:
    def __init__(self, node):
        self.node = node

    # ------------------------------------------------------------------ operators
    def _bin(self, op, other, swap=False):
        o = _wrap(other)
        return Column(("bin", op, o.node, self.node) if swap else ("bin", op, self.node, o.node))

    def __add__(self, o): return self._bin("+", o)
    def __radd__(self, o): return self._bin("+", o, True)
    def __sub__(self, o): return self._bin("-", o)
    def __rsub__(self, o): return self._bin("-", o, True)
    def __mul__(self, o): return self._bin("*", o)
    def __rmul__(self, o): return self._bin("*", o, True)
    def __truediv__(self, o): return self._bin("/", o)
    def __rtruediv__(self, o): return self._bin("/", o, True)
    def __mod__(self, o): return self._bin("%", o)
    def __pow__(self, o): return self._bin("pow", o)
    def __eq__(self, o): return self._bin("==", o)  # noqa: E704
    def __ne__(self, o): return self._bin("!=", o)
    def __lt__(self, o): return self._bin("<", o)
    def __le__(self, o): return self._bin("<=", o)
    def __gt__(self, o): return self._bin(">", o)
    def __ge__(self, o): return self._bin(">=", o)
    def __and__(self, o): return self._bin("&", o)
    def __rand__(self, o): return self._bin("&", o, True)
    def __or__(self, o): return self._bin("|", o)
    def __ror__(self, o): return self._bin("|", o, True)
    def __invert__(self): return Column(("un", "NOT", self.node))
    def __neg__(self): return Column(("un", "NEG", self.node))
    __hash__ = object.__hash__

    def eqNullSafe(self, o): return self._bin("<=>", o)  # noqa: N802
    def isNull(self): return Column(("un", "ISNULL", self.node))  # noqa: N802
    def isNotNull(self): return Column(("un", "ISNOTNULL", self.node))  # noqa: N802
    def isNaN(self): return Column(("un", "ISNAN", self.node))  # noqa: N802

    def isin(self, *vals):
        if len(vals) == 1 and isinstance(vals[0], (list, tuple, set)):
            vals = tuple(vals[0])
        out = None
        for v in vals:
            c = self == v
            out = c if out is None else (out | c)
        return out if out is not None else Column(("lit", False))

    def between(self, lo, hi):
        return (self >= lo) & (self <= hi)

    def alias(self, name: str) -> "Column":
        return Column(("alias", name, self.node))

    name = alias

    def cast(self, dt) -> "Column":
        if isinstance(dt, str):
            dt = {"int": T.IntegerType(), "integer": T.IntegerType(), "long": T.LongType(), "bigint": T.LongType(),
                  "double": T.DoubleType(), "float": T.FloatType(), "boolean": T.BooleanType(),
                  "string": T.StringType()}[dt.lower()]
        return Column(("cast", dt, self.node))

    astype = cast

    def when(self, cond, value) -> "Column":
        if self.node[0] != "when":
            raise TypeError("when() can only be chained on a when() column")
        return Column(("when", self.node[1] + [(_wrap(cond).node, _wrap(value).node)], None))

    def otherwise(self, value) -> "Column":
        if self.node[0] != "when":
            raise TypeError("otherwise() can only be applied on a when() column")
        return Column(("when", self.node[1], _wrap(value).node))

    def asc(self): return Column(("sort", True, self.node))
    def desc(self): return Column(("sort", False, self.node))

    def __repr__(self):
        return f"Column<'{expr_name(self.node)}'>"

    def __bool__(self):
        raise ValueError("Cannot convert column into bool: use '&' for 'and', '|' for 'or', '~' for 'not'")


def col(name: str) -> Column:
    return Column(("col", name))


def lit(v) -> Column:
    return Column(("lit", v))


def expr_name(node) -> str:
    k = node[0]
    if k == "col":
        return node[1]
    if k == "lit":
        return "NULL" if node[1] is None else str(node[1])
    if k == "alias":
        return node[1]
    if k == "bin":
        sym = node[1]
        if sym in ("pow", "least", "greatest", "coalesce"):
            return f"{sym}({expr_name(node[2])}, {expr_name(node[3])})"
        return f"({expr_name(node[2])} {'AND' if sym == '&' else 'OR' if sym == '|' else sym} {expr_name(node[3])})"
    if k == "un":
        op, x = node[1], expr_name(node[2])
        return {"NOT": f"(NOT {x})", "NEG": f"(- {x})", "ISNULL": f"({x} IS NULL)",
                "ISNOTNULL": f"({x} IS NOT NULL)", "ISNAN": f"isnan({x})"}.get(op, f"{op.lower()}({x})")
    if k == "when":
        s = "CASE " + " ".join(f"WHEN {expr_name(c)} THEN {expr_name(v)}" for c, v in node[1])
        if node[2] is not None:
            s += f" ELSE {expr_name(node[2])}"
        return s + " END"
    if k == "cast":
        return f"CAST({expr_name(node[2])} AS {node[1].simple.upper()})"
    if k == "agg":
        fn, x = node[1], node[2]
        return f"{fn}({'1' if x is None else expr_name(x)})" if fn != "count" or x is not None else "count(1)"
    if k == "sort":
        return expr_name(node[2])
    if k == "star":
        return "*"
    return str(node)


def strip_alias(node):
    while node[0] == "alias":
        node = node[2]
    return node


def referenced_columns(node, out=None):
    out = set() if out is None else out
    if node is None:
        return out
    k = node[0]
    if k == "col":
        out.add(node[1])
    elif k in ("bin",):
        referenced_columns(node[2], out); referenced_columns(node[3], out)
    elif k in ("un", "alias", "cast", "sort"):
        referenced_columns(node[2], out)
    elif k == "when":
        for c, v in node[1]:
            referenced_columns(c, out); referenced_columns(v, out)
        referenced_columns(node[2], out)
    elif k == "agg":
        referenced_columns(node[2], out)
    return out


# ------------------------------------------------------------------------------------------------
# type inference
# ------------------------------------------------------------------------------------------------
def _lit_type(v):
    if v is None:
        return T.DoubleType()
    if isinstance(v, bool):
        return T.BooleanType()
    if isinstance(v, int):
        return T.IntegerType() if -2 ** 31 <= v < 2 ** 31 else T.LongType()
    if isinstance(v, float):
        return T.DoubleType()
    if isinstance(v, str):
        return T.StringType()
    raise TypeError(f"unsupported literal {v!r}")


def _wider(a, b):
    order = [T.BooleanType, T.IntegerType, T.LongType, T.FloatType, T.DoubleType]
    ia = next((i for i, c in enumerate(order) if isinstance(a, c)), 4)
    ib = next((i for i, c in enumerate(order) if isinstance(b, c)), 4)
    return order[max(ia, ib, 1)]()


def infer_type(node, table) -> T.DataType:
    k = node[0]
    if k == "col":
        return table.column(node[1]).dtype
    if k == "lit":
        return _lit_type(node[1])
    if k in ("alias", "sort"):
        return infer_type(node[2], table)
    if k == "cast":
        return node[1]
    if k == "un":
        if node[1] in BOOL_OUT:
            return T.BooleanType()
        if node[1] in ("SQRT", "LOG", "EXP"):
            return T.DoubleType()
        return infer_type(node[2], table)
    if k == "bin":
        op = BIN[node[1]]
        if op in BOOL_OUT:
            return T.BooleanType()
        a, b = infer_type(node[2], table), infer_type(node[3], table)
        if op in ("DIV", "POW"):
            return T.DoubleType()
        if isinstance(a, T.StringType) and isinstance(b, T.StringType) and op == "COALESCE":
            return T.StringType()
        return _wider(a, b)
    if k == "when":
        ts = [infer_type(v, table) for _, v in node[1]]
        if node[2] is not None and not (node[2][0] == "lit" and node[2][1] is None):
            ts.append(infer_type(node[2], table))
        out = ts[0]
        for t in ts[1:]:
            out = out if type(out) is type(t) else _wider(out, t)
        return out
    raise TypeError(f"cannot infer type of {node!r}")


# ------------------------------------------------------------------------------------------------
# device compilation
# ------------------------------------------------------------------------------------------------
class _Compiler:
    def __init__(self, table):
        self.table = table
        self.ins: list = []
        self.consts: list = []
        self.cols: list = []
        self.colmap: dict = {}
        self.free = list(range(7, -1, -1))

    def reg(self):
        if not self.free:
            raise ValueError("expression too deep for the device VM (8 registers)")
        return self.free.pop()

    def release(self, r):
        self.free.append(r)

    def const(self, v) -> int:
        self.consts.append(float(v))
        return len(self.consts) - 1

    def column(self, name) -> int:
        if name not in self.colmap:
            from ..ops.df import CT_CODE, TORCH_CT

            cv = self.table.column(name)
            if isinstance(cv.dtype, T.VectorUDT):
                raise TypeError("vector columns are not valid in scalar expressions")
            t = cv.data if cv.data.dtype != torch.bool else cv.data.view(torch.uint8)
            code = CT_CODE if isinstance(cv.dtype, T.StringType) else TORCH_CT[t.dtype]
            self.cols.append((t, cv.valid_u8(), code))
            self.colmap[name] = len(self.cols) - 1
        return self.colmap[name]

    def emit(self, op, d, a=0, b=0, c=0, k=0):
        from ..ops.df import pack_ins

        self.ins.append(pack_ins(op, d, a, b, c, k))

    def string_code(self, colnode, litval):
        """Literal string compared against a dictionary-encoded column -> its code (or -2)."""
        cv = self.table.column(colnode[1])
        lut = cv.dict_index()
        return lut.get(litval, -2)

    def compile(self, node) -> int:
        k = node[0]
        if k == "col":
            r = self.reg()
            self.emit("LDCOL", r, k=self.column(node[1]))
            return r
        if k == "lit":
            r = self.reg()
            v = node[1]
            if v is None:
                self.emit("LDNULL", r)
            elif isinstance(v, str):
                raise TypeError("string literal outside a comparison with a string column")
            else:
                self.emit("LDC", r, k=self.const(float(v)))
            return r
        if k in ("alias", "sort"):
            return self.compile(node[2])
        if k == "cast":
            r = self.compile(node[2])
            if isinstance(node[1], (T.IntegerType, T.LongType)):
                self.emit("CAST_INT", r, r)
            return r
        if k == "un":
            a = self.compile(node[2])
            self.emit(node[1], a, a)
            return a
        if k == "bin":
            op = BIN[node[1]]
            l, rn = node[2], node[3]
            # string column vs string literal -> code comparison
            for x, y in ((l, rn), (rn, l)):
                if x[0] == "col" and y[0] == "lit" and isinstance(y[1], str):
                    if op not in ("EQ", "NE", "EQ_NULLSAFE"):
                        raise TypeError("only equality comparisons are supported on string columns")
                    a = self.compile(x)
                    b = self.reg()
                    self.emit("LDC", b, k=self.const(self.string_code(x, y[1])))
                    self.emit(op, a, a, b)
                    self.release(b)
                    return a
            a = self.compile(l)
            b = self.compile(rn)
            self.emit(op, a, a, b)
            self.release(b)
            return a
        if k == "when":
            # fold from the last branch: res = otherwise; for (c, v) reversed: res = c ? v : res
            other = node[2] if node[2] is not None else ("lit", None)
            res = self.compile(other)
            for cnode, vnode in reversed(node[1]):
                c = self.compile(cnode)
                v = self.compile(vnode)
                self.emit("SELECT", res, c, v, res)
                self.release(v)
                self.release(c)
            return res
        raise TypeError(f"cannot compile {node!r} for the device VM")


def compile_vm(node, table):
    c = _Compiler(table)
    r = c.compile(node)
    return c.ins, r, c.consts, c.cols


# ------------------------------------------------------------------------------------------------
# host (CPU) evaluation with identical semantics
# ------------------------------------------------------------------------------------------------
def eval_host(node, table):
    """-> (float64 values, bool valid) torch CPU tensors."""
    k = node[0]
    n = table.num_rows
    if k == "col":
        cv = table.column(node[1])
        v = cv.data.double() if not isinstance(cv.dtype, T.StringType) else cv.data.double()
        valid = cv.valid_bool()
        if isinstance(cv.dtype, T.StringType):
            valid = valid & (cv.data >= 0)
        return v, valid
    if k == "lit":
        if node[1] is None:
            return torch.zeros(n, dtype=torch.float64), torch.zeros(n, dtype=torch.bool)
        if isinstance(node[1], str):
            raise TypeError("string literal outside a comparison with a string column")
        return torch.full((n,), float(node[1]), dtype=torch.float64), torch.ones(n, dtype=torch.bool)
    if k in ("alias", "sort"):
        return eval_host(node[2], table)
    if k == "cast":
        v, ok = eval_host(node[2], table)
        if isinstance(node[1], (T.IntegerType, T.LongType)):
            ok = ok & ~torch.isnan(v)
            v = torch.trunc(v)
        return v, ok
    if k == "un":
        v, ok = eval_host(node[2], table)
        op = node[1]
        one, zero = torch.ones_like(v), torch.zeros_like(v)
        if op == "NOT":
            return torch.where(v == 0, one, zero), ok
        if op == "NEG":
            return -v, ok
        if op == "ISNULL":
            return (~ok).double(), torch.ones_like(ok)
        if op == "ISNOTNULL":
            return ok.double(), torch.ones_like(ok)
        if op == "ISNAN":
            return (ok & torch.isnan(v)).double(), torch.ones_like(ok)
        f = {"ABS": torch.abs, "SQRT": torch.sqrt, "EXP": torch.exp, "FLOOR": torch.floor, "CEIL": torch.ceil,
             "ROUND": torch.round, "LOG": torch.log}[op]
        out = f(v)
        if op == "LOG":
            ok = ok & (v > 0)
        return out, ok
    if k == "bin":
        op = BIN[node[1]]
        l, rn = node[2], node[3]
        for x, y in ((l, rn), (rn, l)):
            if x[0] == "col" and y[0] == "lit" and isinstance(y[1], str):
                cv = table.column(x[1])
                code = cv.dict_index().get(y[1], -2)
                a, va = eval_host(x, table)
                b = torch.full_like(a, float(code))
                return _bin_host(op, a, va, b, torch.ones_like(va))
        a, va = eval_host(l, table)
        b, vb = eval_host(rn, table)
        return _bin_host(op, a, va, b, vb)
    if k == "when":
        other = node[2] if node[2] is not None else ("lit", None)
        res, rv = eval_host(other, table)
        for cnode, vnode in reversed(node[1]):
            c, vc = eval_host(cnode, table)
            v, vv = eval_host(vnode, table)
            t = vc & (c != 0)
            res = torch.where(t, v, res)
            rv = torch.where(t, vv, rv)
        return res, rv
    raise TypeError(f"cannot evaluate {node!r}")


def _bin_host(op, a, va, b, vb):
    one, zero = torch.ones_like(a), torch.zeros_like(a)
    both = va & vb
    if op == "ADD":
        return a + b, both
    if op == "SUB":
        return a - b, both
    if op == "MUL":
        return a * b, both
    if op == "DIV":
        return a / torch.where(b == 0, one, b), both & (b != 0)
    if op == "MOD":
        return torch.fmod(a, torch.where(b == 0, one, b)), both & (b != 0)
    if op == "POW":
        return torch.pow(a, b), both
    if op in ("EQ", "NE"):
        eq = (a == b) | (torch.isnan(a) & torch.isnan(b))
        return torch.where(eq if op == "EQ" else ~eq, one, zero), both
    if op == "LT":
        return (a < b).double(), both
    if op == "LE":
        return (a <= b).double(), both
    if op == "GT":
        return (a > b).double(), both
    if op == "GE":
        return (a >= b).double(), both
    if op == "AND":
        fa, fb = va & (a == 0), vb & (b == 0)
        f = fa | fb
        return torch.where(f, zero, one), f | both
    if op == "OR":
        ta, tb = va & (a != 0), vb & (b != 0)
        t = ta | tb
        return torch.where(t, one, zero), t | both
    if op == "EQ_NULLSAFE":
        return torch.where(both, (a == b).double(), (va == vb).double()), torch.ones_like(va)
    if op == "MIN2":
        return torch.fmin(a, b), both
    if op == "MAX2":
        return torch.fmax(a, b), both
    if op == "COALESCE":
        return torch.where(va, a, b), va | vb
    raise TypeError(op)


_ = math
