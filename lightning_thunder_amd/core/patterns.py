"""Pattern matching over traces (reference ``thunder/core/patterns.py``: ``Pattern``, ``match_all``,
``bind_names``, ``numbered_ancestors``).

A :class:`Pattern` is a sequence of steps.  Each step has

* a **matcher** on a bound symbol, returning ``bool`` or ``(bool, ctx_update)``: the dict updates
  a per-match context that later steps see (e.g. "the weight of the linear I matched");
* an optional **condition** ``condition(previous_bsyms, bsym[, ctx])`` on the earlier matches;
* a repetition range ``min_times .. max_times`` (``max_times=-1``: unbounded) — a repeated step
  matches consecutive dataflow-connected symbols greedily;
* ``connected``: whether the symbol must consume an output of the partial match (the default), or
  may be any later symbol that can be *reordered next to the match* — it must not depend on a
  symbol between the match and itself that depends on the partial match.

Symbols skipped between matched ones must not depend on the partial match, so the matched group can
be replaced at the position of its last member.  :func:`match_all` returns non-overlapping matches
as lists of ``(index, bsym)``; ``Pattern.contexts`` holds each match's context dict.  Used by
transforms that rewrite idioms (e.g. fusing ``linear`` + bias + activation epilogues).
"""
from __future__ import annotations

import inspect
from typing import Any, Callable

from .symbol import BoundSymbol
from .trace import TraceCtx

_SKIPPABLE = ("python_del", "comment")


def bind_names(bsym: BoundSymbol) -> dict[str, Any]:
    """The bound symbol's inputs by parameter name (``bind_names(b)["weight"]``), from the
    signature of the symbol's meta / Python implementation; positional extras become ``arg<i>``."""
    fn = getattr(bsym.sym, "meta", None) or getattr(bsym.sym, "fn", None)
    try:
        sig = inspect.signature(fn)
        ba = sig.bind_partial(*bsym.args, **bsym.kwargs)
        out = dict(ba.arguments)
        for k, p in sig.parameters.items():
            if p.kind is inspect.Parameter.VAR_POSITIONAL and k in out:
                out.update({f"arg{i}": v for i, v in enumerate(out.pop(k), start=len(out))})
            elif p.kind is inspect.Parameter.VAR_KEYWORD and k in out:
                out.update(out.pop(k))
        return out
    except (TypeError, ValueError):
        out = {f"arg{i}": a for i, a in enumerate(bsym.args)}
        out.update(bsym.kwargs)
        return out


def numbered_ancestors(trace: TraceCtx) -> list[set[int]]:
    """Per bound symbol: the indices of ALL its producers (transitively)."""
    prod: dict[str, int] = {}
    anc: list[set[int]] = []
    for i, b in enumerate(trace.bound_symbols):
        s: set[int] = set()
        for a in b.flat_proxy_args:
            j = prod.get(a.name)
            if j is not None:
                s.add(j)
                s |= anc[j]
        anc.append(s)
        for o in b.flat_proxy_outs:
            prod[o.name] = i
    return anc


_ancestors = numbered_ancestors  # back-compat name


def _call_matcher(m, b) -> tuple[bool, dict]:
    r = m(b)
    if isinstance(r, tuple):
        ok, upd = r
        return bool(ok), dict(upd or {})
    return bool(r), {}


def _call_condition(cond, prev, b, ctx) -> bool:
    if cond is None:
        return True
    try:
        n = len(inspect.signature(cond).parameters)
    except (TypeError, ValueError):
        n = 2
    return bool(cond(prev, b, ctx) if n >= 3 else cond(prev, b))


class Pattern:
    def __init__(self):
        # (matcher, condition, min_times, max_times, connected)
        self.steps: list[tuple[Callable, Callable | None, int, int, bool]] = []
        self.contexts: list[dict] = []

    def match(self, matcher: Callable, condition: Callable | None = None, *, min_times: int = 1, max_times: int = 1,
              connected: bool = True) -> "Pattern":
        """Adds a step (see the module docstring); returns ``self`` for chaining."""
        if min_times < 0 or (max_times != -1 and max_times < max(min_times, 1)):
            raise ValueError(f"bad repetition range {min_times}..{max_times}")
        self.steps.append((matcher, condition, min_times, max_times, connected))
        return self

    def __call__(self, trace: TraceCtx) -> list[list[tuple[int, BoundSymbol]]]:
        return match_all(trace, self)


def _independent_of_partial(bsyms, anc, lo: int, hi: int, idxs: set[int]) -> bool:
    """No unmatched, non-trivial symbol in (lo, hi) depends on the partial match ``idxs``."""
    for k in range(lo + 1, hi):
        if k in idxs or bsyms[k].sym.name in _SKIPPABLE:
            continue
        if anc[k] & idxs:
            return False
    return True


def match_all(trace: TraceCtx, pattern: Pattern) -> list[list[tuple[int, BoundSymbol]]]:
    """Non-overlapping matches of ``pattern`` in ``trace`` (lists of ``(index, bsym)``)."""
    bsyms = trace.bound_symbols
    anc = numbered_ancestors(trace)
    used: set[int] = set()
    results: list[list[tuple[int, BoundSymbol]]] = []
    pattern.contexts = []
    if not pattern.steps:
        return results

    def candidates(after: int, matched: list[tuple[int, BoundSymbol]], produced: set[str], connected: bool,
                   consecutive: bool):
        idxs = {m[0] for m in matched}
        first = matched[0][0] if matched else after
        for j in range(after + 1, len(bsyms)):
            if j in used:
                continue
            c = bsyms[j]
            if c.sym.name in _SKIPPABLE:
                continue
            if connected and matched and not any(a.name in produced for a in c.flat_proxy_args):
                if consecutive:
                    return  # a repeated step matches consecutive symbols only
                continue
            if matched and not _independent_of_partial(bsyms, anc, first, j, idxs):
                return  # later symbols would have to move across a consumer of the partial match
            yield j, c
            if consecutive:
                return

    def step_matches(si: int, matched, produced, ctx, after: int):
        """All ways (greedy first) to satisfy steps[si:], as (matched, ctx)."""
        if si == len(pattern.steps):
            yield matched, ctx
            return
        m, cond, lo, hi, connected = pattern.steps[si]
        # greedy repetition: collect up to `hi` consecutive matches, then back off to `lo`
        chain: list[tuple[int, BoundSymbol, dict]] = []
        cur_matched, cur_produced, cur_ctx, cur_after = list(matched), set(produced), dict(ctx), after
        states = [(list(cur_matched), set(cur_produced), dict(cur_ctx), cur_after)]
        while hi == -1 or len(chain) < hi:
            found = None
            for j, c in candidates(cur_after, cur_matched, cur_produced, connected, consecutive=bool(chain)):
                ok, upd = _call_matcher(m, c)
                if ok and _call_condition(cond, [x[1] for x in cur_matched], c, {**cur_ctx, **upd}):
                    found = (j, c, upd)
                    break
            if found is None:
                break
            j, c, upd = found
            chain.append(found)
            cur_matched = cur_matched + [(j, c)]
            cur_produced = cur_produced | {o.name for o in c.flat_proxy_outs}
            cur_ctx = {**cur_ctx, **upd}
            cur_after = j
            states.append((list(cur_matched), set(cur_produced), dict(cur_ctx), cur_after))
        for n in range(len(chain), lo - 1, -1):
            if n == 0 and lo > 0:
                break
            sm, sp, sc, sa = states[n]
            yield from step_matches(si + 1, sm, sp, sc, sa)

    for start in range(len(bsyms)):
        if start in used or bsyms[start].sym.name in _SKIPPABLE:
            continue
        m0, cond0, lo0, hi0, _ = pattern.steps[0]
        ok, upd = _call_matcher(m0, bsyms[start])
        if not ok or not _call_condition(cond0, [], bsyms[start], upd):
            continue
        # the first step's remaining repetitions continue from `start`
        first = [(start, bsyms[start])]
        produced = {o.name for o in bsyms[start].flat_proxy_outs}
        saved = pattern.steps[0]
        rest_lo, rest_hi = max(lo0 - 1, 0), (hi0 - 1 if hi0 != -1 else -1)
        try:
            if rest_hi != 0:
                pattern.steps[0] = (m0, cond0, rest_lo, rest_hi, saved[4])
                it = step_matches(0, first, produced, upd, start)
            else:
                it = step_matches(1, first, produced, upd, start)
            res = next(iter(it), None)
        finally:
            pattern.steps[0] = saved
        if res is None:
            continue
        matched, ctx = res
        results.append(matched)
        pattern.contexts.append(ctx)
        used |= {i for i, _ in matched}
    return results
