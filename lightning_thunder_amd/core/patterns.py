"""Pattern matching over traces (reference ``thunder/core/patterns.py``: ``Pattern``, ``match_all``).

A :class:`Pattern` is a sequence of steps; each step is a predicate on a bound symbol (usually
"is symbol X") plus optional conditions on the previously matched symbols.  Matches must be
dataflow-connected in order (each matched symbol consumes an output of an earlier match) and
may skip unrelated bound symbols in between, as long as the skipped ones do not depend on the
partial match (so the matched group can be replaced at the position of its last member).
Used by transforms that rewrite idioms (e.g. fusing ``linear`` + bias + activation epilogues).
"""
from __future__ import annotations

from typing import Callable

from .symbol import BoundSymbol
from .trace import TraceCtx


def _ancestors(trace: TraceCtx) -> list[set[int]]:
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


class Pattern:
    def __init__(self):
        self.steps: list[tuple[Callable[[BoundSymbol], bool], Callable | None]] = []

    def match(self, predicate: Callable[[BoundSymbol], bool], condition: Callable | None = None) -> "Pattern":
        """Adds a step; ``condition(previous_matches, bsym)`` may inspect the earlier matches."""
        self.steps.append((predicate, condition))
        return self

    def __call__(self, trace: TraceCtx) -> list[list[tuple[int, BoundSymbol]]]:
        return match_all(trace, self)


def match_all(trace: TraceCtx, pattern: Pattern) -> list[list[tuple[int, BoundSymbol]]]:
    """Non-overlapping matches of ``pattern`` in ``trace`` (lists of (index, bsym))."""
    bsyms = trace.bound_symbols
    anc = _ancestors(trace)
    used: set[int] = set()
    results = []
    for start, b in enumerate(bsyms):
        if start in used or not pattern.steps:
            continue
        pred, cond = pattern.steps[0]
        if not pred(b) or (cond is not None and not cond([], b)):
            continue
        matched = [(start, b)]
        produced = {o.name for o in b.flat_proxy_outs}
        ok = True
        i = start
        for pred, cond in pattern.steps[1:]:
            found = None
            for j in range(i + 1, len(bsyms)):
                if j in used:
                    continue
                c = bsyms[j]
                if pred(c) and any(a.name in produced for a in c.flat_proxy_args) and \
                        (cond is None or cond([m[1] for m in matched], c)):
                    found = j
                    break
            if found is None:
                ok = False
                break
            # nothing between the first match and `found` that is not matched may consume the partial match
            idxs = {m[0] for m in matched}
            for k in range(start + 1, found):
                if bsyms[k].sym.name in ("python_del", "comment"):
                    continue
                if k not in idxs and anc[k] & idxs:
                    ok = False
                    break
            if not ok:
                break
            matched.append((found, bsyms[found]))
            produced |= {o.name for o in bsyms[found].flat_proxy_outs}
            i = found
        if ok:
            results.append(matched)
            used |= {m[0] for m in matched}
    return results
