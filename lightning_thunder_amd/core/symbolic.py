"""Symbolic tensor dims for ``cache="symbolic values"`` (parity: the reference's symbolic tensor shapes,
``thunder/core/proxies.py:1271-1274,1490-1495,2015-2020`` and ``thunder/core/jit_ext.py:289-291``).

Design.  A dim of a non-parameter tensor argument becomes a :class:`SymInt`: an ``int`` subclass that
carries the value seen while tracing AND an expression over the call's dim symbols (``s0``, ``s1`` ...).
Because it *is* an int, every meta function, VJP rule and executor checker keeps working unchanged;
what changes is what is remembered:

* arithmetic (``+ - * // %``, ``math.prod``, negation) returns a new SymInt whose expression is the
  arithmetic, so a ``reshape(a, [a.numel()])`` prints as ``reshape(a, [(s0 * s1)])`` in the program;
* a comparison, ``bool()`` or ``min``/``max`` returns a plain bool and records a *guard* (the expression
  and the outcome seen), e.g. the broadcasting rule's ``s0 == 1`` records ``s0 != 1``;
* anything that needs the bare value — ``int()``, ``__index__`` (``range``, list indexing, a real torch
  call), ``float()``, ``str``/``format`` — *specializes*: it records ``expr == value``.

The guards are evaluated against the new call's dims after the prologue's rank / dtype / device checks,
so one cache entry serves every size that takes the same path through the program, and correctness
never depends on a dim the program did not prove it can vary.  Dims of size 0 and 1 are not made
symbolic (PyTorch's 0/1 specialization; broadcasting depends on them).

Generated programs bind the symbols they print from their own tensor arguments (``s0 = t_x.shape[1]``);
a program whose arguments do not carry a symbol prints its value and specializes on it instead.
Heuristic code (rematerialization cut weights, fusion cost models) runs under :func:`no_guards`, because
their decisions are valid for any size.  Known gap (recorded, not guarded): ``float op SymInt`` with the
float on the LEFT goes through ``float.__mul__`` and never reaches this class.
"""
from __future__ import annotations

import contextlib
import operator
from contextvars import ContextVar
from typing import Any, Callable

_env: ContextVar = ContextVar("lta_shape_env", default=None)


class ShapeEnv:
    """Symbols, guards and specializations of one compilation."""

    def __init__(self):
        self.symbols: list[tuple[str, int, int, int]] = []  # (name, flat-arg index, dim, traced value)
        self.guards: dict[str, bool] = {}
        self._suspended = 0
        self._parent: dict[str, str] = {}

    # -- symbols ---------------------------------------------------------------------------------
    def new_symbol(self, value: int, arg_index: int, dim: int | None) -> "SymInt":
        """A symbol for dim ``dim`` of tensor argument ``arg_index`` (``dim=None``: the int argument itself)."""
        name = f"s{len(self.symbols)}"
        self.symbols.append((name, arg_index, dim, int(value)))
        self._parent[name] = name
        return SymInt(value, name)

    # -- equal symbols (a recorded ``s3 == s1``): a program that cannot bind one binds the other --------
    def _find(self, a: str) -> str:
        while self._parent.get(a, a) != a:
            a = self._parent[a]
        return a

    def equivalents(self, name: str) -> list[str]:
        r = self._find(name)
        return [n for n in self._parent if self._find(n) == r]

    @property
    def active(self) -> bool:
        return self._suspended == 0

    def record(self, expr: str, outcome: bool) -> None:
        if self._suspended:
            return
        self.guards[expr] = bool(outcome)
        parts = expr.split(" == ")
        if outcome and len(parts) == 2 and all(p in self._parent for p in parts):
            self._parent[self._find(parts[0])] = self._find(parts[1])

    def specialize(self, s: "SymInt") -> None:
        self.record(f"({s.expr}) == {int.__int__(s)}", True)

    # -- the guard function --------------------------------------------------------------------------
    def guard_source(self) -> str:
        conds = [(e if ok else f"not ({e})") for e, ok in self.guards.items()]
        return " and ".join(f"({c})" for c in conds) if conds else "True"

    def guard_fn(self) -> Callable[[list], bool]:
        """``check(flat_args) -> bool``: binds every symbol from the call's arguments and evaluates the
        recorded guards (compiled once)."""
        names = [n for n, _, _, _ in self.symbols]
        src = f"def _guards({', '.join(names)}):\n  return {self.guard_source()}\n"
        ns: dict[str, Any] = {}
        exec(compile(src, "<lta symbolic guards>", "exec"), ns)
        g = ns["_guards"]
        where = [(i, d) for _, i, d, _ in self.symbols]

        def check(flat_args):
            return bool(g(*[flat_args[i] if d is None else flat_args[i].shape[d] for i, d in where]))

        check.source = src
        return check


def current_env() -> ShapeEnv | None:
    return _env.get()


@contextlib.contextmanager
def shape_env(env: ShapeEnv | None):
    tok = _env.set(env)
    try:
        yield env
    finally:
        _env.reset(tok)


@contextlib.contextmanager
def no_guards():
    """Comparisons of symbolic dims inside this block record nothing (size heuristics whose outcome is
    valid for every size: cost models, cut weights, logging)."""
    env = _env.get()
    if env is None:
        yield
        return
    env._suspended += 1
    try:
        yield
    finally:
        env._suspended -= 1


def _expr(x) -> str:
    return x.expr if isinstance(x, SymInt) else repr(int(x))


def _record(expr: str, outcome: bool) -> bool:
    env = _env.get()
    if env is not None:
        env.record(expr, outcome)
    return outcome


def _specialize(s: "SymInt") -> int:
    env = _env.get()
    if env is not None:
        env.specialize(s)
    return int.__int__(s)


def _plain(x) -> bool:
    return type(x) is int or isinstance(x, SymInt)


class SymInt(int):
    """An int that remembers how it was computed from the call's symbolic dims (module docstring)."""

    def __new__(cls, value: int, expr: str, poly: dict | None = None):
        self = int.__new__(cls, int(value))
        # poly: {monomial (sorted tuple of atoms): coefficient}; a bare symbol is {("s0",): 1}
        self.poly = poly if poly is not None else {(expr,): 1}
        self.expr = expr
        return self

    # -- introspection -----------------------------------------------------------------------------
    @property
    def value(self) -> int:
        return int.__int__(self)

    def free_symbols(self) -> set[str]:
        import re

        return set(re.findall(r"\bs\d+\b", self.expr))

    def __call__(self):  # ``TensorProxy.numel`` is callable as well as an int (reference parity)
        return self

    # -- value reads specialize ----------------------------------------------------------------------
    def __index__(self):
        return _specialize(self)

    def __int__(self):
        return _specialize(self)

    def __float__(self):
        return float(_specialize(self))

    def __repr__(self):
        return repr(_specialize(self))

    __str__ = __repr__

    def __format__(self, spec):
        return format(_specialize(self), spec)

    def __bool__(self):
        return _record(f"({self.expr}) != 0", int.__int__(self) != 0)

    def __hash__(self):
        return int.__hash__(self)

    def __reduce__(self):
        return (int, (int.__int__(self),))

    # -- arithmetic stays symbolic ------------------------------------------------------------------
    # Expressions are kept as integer polynomials over atoms (a symbol, or an opaque ``(p // c)`` /
    # ``(p % c)`` term) in a canonical form, so ``(s0 - s0) + s0`` IS ``s0`` and a product written two
    # ways compares identical: the guards stay short and identities record nothing.
    def __add__(self, o):
        return _arith(self, o, "+")

    def __radd__(self, o):
        return _arith(o, self, "+")

    def __sub__(self, o):
        return _arith(self, o, "-")

    def __rsub__(self, o):
        return _arith(o, self, "-")

    def __mul__(self, o):
        return _arith(self, o, "*")

    def __rmul__(self, o):
        return _arith(o, self, "*")

    def __floordiv__(self, o):
        return _arith(self, o, "//")

    def __rfloordiv__(self, o):
        return _arith(o, self, "//")

    def __mod__(self, o):
        return _arith(self, o, "%")

    def __rmod__(self, o):
        return _arith(o, self, "%")

    def __divmod__(self, o):
        return self // o, self % o

    def __truediv__(self, o):
        return _specialize(self) / (int(o) if isinstance(o, SymInt) else o)

    def __rtruediv__(self, o):
        return (int(o) if isinstance(o, SymInt) else o) / _specialize(self)

    def __pow__(self, o, mod=None):
        if mod is None and type(o) is int and 0 <= o <= 4:
            r = 1
            for _ in range(o):
                r = r * self
            return r
        return pow(_specialize(self), int(o) if isinstance(o, SymInt) else o, mod)

    def __rpow__(self, o):
        return pow(o, _specialize(self))

    def __neg__(self):
        return _arith(0, self, "-")

    def __pos__(self):
        return self

    def __abs__(self):
        return self if self >= 0 else -self

    def __trunc__(self):
        return self

    __floor__ = __ceil__ = __trunc__

    def __round__(self, ndigits=None):
        return self if ndigits is None else _specialize(self)

    def __and__(self, o):
        return _specialize(self) & o

    __rand__ = __and__

    def __or__(self, o):
        return _specialize(self) | o

    __ror__ = __or__

    def __xor__(self, o):
        return _specialize(self) ^ o

    __rxor__ = __xor__

    def __lshift__(self, o):
        return _specialize(self) << o

    def __rshift__(self, o):
        return _specialize(self) >> o

    def __invert__(self):
        return ~_specialize(self)

    # -- comparisons record guards -------------------------------------------------------------------
    def _cmp(self, other, op: str, fn):
        if isinstance(other, bool) or not _plain(other):
            if isinstance(other, float):
                return fn(_specialize(self), other)
            return NotImplemented
        a = int.__int__(self)
        b = int.__int__(other) if isinstance(other, SymInt) else other
        out = fn(a, b)
        diff = _padd(self.poly, _poly_of(other), -1)
        if not diff or list(diff) == [()]:
            return out  # the two sides differ by a constant: the outcome holds for every size
        return _record(f"{self.expr} {op} {_expr(other)}", out)

    def __eq__(self, o):
        return self._cmp(o, "==", lambda a, b: a == b)

    def __ne__(self, o):
        return self._cmp(o, "!=", lambda a, b: a != b)

    def __lt__(self, o):
        return self._cmp(o, "<", lambda a, b: a < b)

    def __le__(self, o):
        return self._cmp(o, "<=", lambda a, b: a <= b)

    def __gt__(self, o):
        return self._cmp(o, ">", lambda a, b: a > b)

    def __ge__(self, o):
        return self._cmp(o, ">=", lambda a, b: a >= b)



# -- canonical integer polynomials over atoms -------------------------------------------------------------
def _poly_of(x) -> dict:
    if isinstance(x, SymInt):
        return x.poly
    return {(): int(x)} if x else {}


def _padd(p: dict, q: dict, sign: int = 1) -> dict:
    r = dict(p)
    for m, c in q.items():
        v = r.get(m, 0) + sign * c
        if v:
            r[m] = v
        else:
            r.pop(m, None)
    return r


def _pmul(p: dict, q: dict) -> dict:
    r: dict = {}
    for m1, c1 in p.items():
        for m2, c2 in q.items():
            m = tuple(sorted(m1 + m2))
            v = r.get(m, 0) + c1 * c2
            if v:
                r[m] = v
            else:
                r.pop(m, None)
    return r


def _pstr(p: dict) -> str:
    if not p:
        return "0"
    terms = []
    for m in sorted(p, key=lambda m: (-len(m), m)):
        c = p[m]
        body = "*".join(m)
        if not m:
            t = repr(abs(c))
        elif abs(c) == 1:
            t = body
        else:
            t = f"{abs(c)}*{body}"
        terms.append(("-" if c < 0 else "+", t))
    out = ("-" if terms[0][0] == "-" else "") + terms[0][1]
    for sg, t in terms[1:]:
        out += f" {sg} {t}"
    return out if len(terms) == 1 and not out.startswith("-") else f"({out})"


def _operand(p: dict) -> str:
    """A polynomial as an operand of ``//`` / ``%``: parenthesized unless it is a single atom."""
    t = _pstr(p)
    return t if t.isidentifier() or (t.startswith("(") and len(p) == 1 and list(p.values()) == [1]
                                     and len(next(iter(p))) == 1) else f"({t})" if not t.startswith("(") else t


def _make(value: int, poly: dict):
    if not poly or list(poly) == [()]:
        return int(value)  # the expression folded to a constant
    if len(poly) == 1:
        (m, c), = poly.items()
        if c == 1 and len(m) == 1:
            return SymInt(value, m[0], poly)
    return SymInt(value, _pstr(poly), poly)


def _arith(a, b, op: str):
    """``a op b`` with at least one SymInt operand (the other an int, a float, or not a number)."""
    for x in (a, b):
        if isinstance(x, float):
            av = _specialize(a) if isinstance(a, SymInt) else a
            bv = _specialize(b) if isinstance(b, SymInt) else b
            return {"+": operator.add, "-": operator.sub, "*": operator.mul, "//": operator.floordiv,
                    "%": operator.mod}[op](av, bv)
        if not isinstance(x, int):
            return NotImplemented  # tensors / number proxies: their reflected operator handles it
    av = int.__int__(a) if isinstance(a, SymInt) else int(a)
    bv = int.__int__(b) if isinstance(b, SymInt) else int(b)
    pa, pb = _poly_of(a), _poly_of(b)
    if op == "+":
        return _make(av + bv, _padd(pa, pb))
    if op == "-":
        return _make(av - bv, _padd(pa, pb, -1))
    if op == "*":
        return _make(av * bv, _pmul(pa, pb))
    val = av // bv if op == "//" else av % bv
    if not isinstance(b, SymInt) and bv > 0:
        if all(c % bv == 0 for c in pa.values()):  # exact: every term is a multiple of the divisor
            return _make(val, {m: c // bv for m, c in pa.items()} if op == "//" else {})
        if bv == 1:
            return a if op == "//" else 0
    atom = f"({_operand(pa) if isinstance(a, SymInt) else repr(av)} {op} {_operand(pb) if isinstance(b, SymInt) else repr(bv)})"
    return SymInt(val, atom, {(atom,): 1})

def is_symbolic(x) -> bool:
    return isinstance(x, SymInt)


def any_symbolic(shape) -> bool:
    return any(isinstance(s, SymInt) for s in shape)


def static_value(x):
    """The traced value without recording anything (for heuristics and cost models)."""
    return int.__int__(x) if isinstance(x, SymInt) else x


class SymShape(tuple):
    """A tensor proxy's shape when some dims are symbolic (``torch.Size`` would turn them into plain
    ints through ``__index__``).  Behaves like ``torch.Size`` for the calls traced code makes."""

    def numel(self):
        n = 1
        for s in self:
            n = n * s
        return n

    def __getitem__(self, k):
        r = tuple.__getitem__(self, k)
        return SymShape(r) if isinstance(k, slice) else r

    def __add__(self, o):
        return SymShape(tuple(self) + tuple(o))

    def __radd__(self, o):
        return SymShape(tuple(o) + tuple(self))

    def __repr__(self):
        return "SymShape([" + ", ".join(s.expr if isinstance(s, SymInt) else repr(s) for s in self) + "])"


def make_shape(shape):
    """``torch.Size`` for static shapes, :class:`SymShape` when any dim is symbolic."""
    import torch

    if any(isinstance(s, SymInt) for s in shape):
        return SymShape(shape)
    return torch.Size(shape)


def unify(a, b):
    """Of two dims already known equal, the symbolic one (so a plain int from one operand does not
    erase the symbol another operand carries)."""
    return b if isinstance(b, SymInt) and not isinstance(a, SymInt) else a


def unify_shapes(a, b) -> tuple:
    return tuple(unify(x, y) for x, y in zip(a, b))
