"""hipfuse: the HIP fusion executor (K1; role of nvFuser in the reference).

Reference parity:
* ``FusionExecutor.fusion_pass`` — ``thunder/executors/nvfuserex_impl.py:794-915`` (flatten
  claimed bound symbols, partition, build fusion regions, name them ``nvFusionN``).
* partitioners — ``thunder/executors/data_dependent_partition.py`` (``consecutive`` /
  ``dataflow``).  The default is dataflow: a Kahn toposort inside each side-effect-free segment
  that keeps scheduling ready bound symbols into the open region as long as the region's
  iteration domain admits them (see ``hipfuse_codegen.Plan``); compile option
  ``fusion_type="consecutive"`` admits only the next bound symbol in program order.
* optimization fuel — ``THUNDER_HIPFUSE_FUEL`` bounds the number of regions created.

Each region becomes one ``hipFusionN`` callable: Python generates HIP source per call
signature (input strides + alignment), the native runtime (``ops/csrc/runtime/rtc.cpp``)
compiles it with hiprtc for gfx950 and launches it on the current HIP stream.  Code
objects are cached in memory and on disk (``$LTA_CACHE_DIR`` or ``ops/_build/rtc_cache``).
"""
from __future__ import annotations

import ctypes
import heapq
import hashlib
import itertools
import os
import threading

from ..core.rng import GraphRngInt

import torch

from ..core.symbolic import SymInt

from ..core import profile as _profile
from ..core.prims import PrimIDs, OpTags
from ..core.proxies import TensorProxy, Proxy
from ..core.pytree import tree_flatten, tree_map
from ..core.symbol import Symbol, BoundSymbol
from ..core.trace import from_trace, TraceProvenance
from ..extend import FusionExecutor, register_executor, add_default_executor
from . import hipfuse_codegen as cg

ex = FusionExecutor("hipfuse")
register_executor(ex)


def _add_after_hipex():
    # default order: hipex (whole-op HIP kernels) claims first, then hipfuse fuses what is left
    from ..extend import _default_executors

    if ex not in _default_executors:
        _default_executors.append(ex)


_add_after_hipex()
ex.allow_cpu = False  # tests flip this to exercise partitioning/codegen on CPU tensors

_counter = itertools.count()


def _checker(*args, **kwargs):
    dev = kwargs.get("device")
    if dev is not None and getattr(dev, "type", None) not in (None, "cuda") and not ex.allow_cpu:
        return False
    for a in tree_flatten((args, kwargs))[0]:
        if isinstance(a, TensorProxy):
            if not cg.supported_dtype(a.dtype):
                return False
            if a.device.type != "cuda" and not ex.allow_cpu:
                return False
            if any(not isinstance(s, int) or isinstance(s, SymInt) for s in a.shape):
                # symbolic dims (cache="symbolic values"): generated kernels bake their sizes in, so
                # these ops stay on the per-op executors and one program serves every size
                return False
    return True


for _sid in cg.SUPPORTED:
    ex.register_supported(_sid, _checker)


def _symbolic(b: BoundSymbol) -> bool:
    return any(isinstance(p, TensorProxy) and any(isinstance(d, SymInt) for d in p._shape)
               for p in (*b.flat_proxy_args, *b.flat_proxy_outs))


def _is_barrier(b: BoundSymbol) -> bool:
    if b.sym.id in (PrimIDs.RETURN, PrimIDs.DEL, PrimIDs.COMMENT):
        return True
    if _symbolic(b):
        return True  # symbolic dims: no region (kernels bake sizes in), not even a view inside one
    tags = set(b.sym.tags or ()) | set(getattr(b, "tags", ()) or ())
    if OpTags.DONT_DCE in tags or OpTags.IN_PLACE in tags or OpTags.RANDOM_OP in tags:
        return True
    return getattr(b.sym, "module", None) == "dist_prims" or (isinstance(b.sym.id, str) and b.sym.id.startswith("dist."))


def _fusible_leaf(b: BoundSymbol) -> bool:
    return b.sym.id in cg.SUPPORTED and ex.can_execute_directly(b)


def _flatten(b: BoundSymbol) -> list:
    if _fusible_leaf(b):
        return [b]
    if b.sym.executor is None and not b.sym.is_fusion and b.subsymbols and ex.can_fuse(b):
        outs = [o.name for o in b.flat_outs]
        flat = []
        for s in b.subsymbols:
            flat.extend(_flatten(s))
        produced = {o.name for s in flat for o in s.flat_outs}
        ins = {a.name for a in b.flat_proxy_args}
        # a decomposition that does not produce its own outputs (e.g. returns an alias) stays whole
        if all(n in produced or n in ins for n in outs) and all(n in produced for n in outs if n not in ins):
            if any(n in ins and n not in produced for n in outs):
                return [b]
            return flat
    return [b]


class HipFusion:
    """Callable for one fusion region (what the trace calls as ``hipFusionN``)."""

    def __init__(self, name: str, plan: cg.Plan, inputs: list, outputs: list, nodes: list):
        self.name = name
        self.plan = plan
        self.inputs = inputs
        self.outputs = outputs
        self.nodes = nodes
        self.tensor_pos = [i for i, a in enumerate(inputs) if isinstance(a, TensorProxy)]
        self.number_pos = [i for i, a in enumerate(inputs) if not isinstance(a, TensorProxy)]
        self._variants: dict = {}
        self._lock = threading.Lock()
        # + the workspace pointer (column mode) in the second type
        self._argbuf_t, self._argbuf_ws_t = arg_buffer_types(len(self.tensor_pos), len(outputs), len(self.number_pos))
        # regions have static shapes (symbolic bound symbols are fusion barriers): the output
        # allocations are fixed once here instead of re-deriving proxy shapes on every call
        self._out_specs = [(tuple(int(d) for d in o.shape), o.dtype) for o in outputs]
        self._out_empty = any(0 in shape for shape, _ in self._out_specs)

    def __repr__(self):
        return f"HipFusion({self.name}, {len(self.nodes)} prims)"

    # -- reference path (CPU tensors; used by CPU tests of partitioning) ----------------------
    def _run_reference(self, args):
        from .torchex import ex as tex

        env = {p.name: a for p, a in zip(self.inputs, args) if isinstance(p, Proxy)}

        def get(x):
            return env.get(x.name, x) if isinstance(x, Proxy) else x

        for b in self.nodes:
            impl = tex.implmap[b.sym.id].symbol.impl_fn
            r = impl(*tree_map(get, b.args), **tree_map(get, b.kwargs))
            outs = b.flat_outs
            vals = tree_flatten(r)[0]
            for o, v in zip(outs, vals):
                env[o.name] = v
        return tuple(env[o.name] for o in self.outputs)

    # -- native path ---------------------------------------------------------------------------
    def _variant(self, tensors, rng_key=()):
        key = tuple((tuple(t.stride()), t.data_ptr() % 16 == 0) for t in tensors)
        if rng_key:
            key = (key, rng_key)
        v = self._variants.get(key)
        if v is not None:
            return v
        with self._lock:
            v = self._variants.get(key)
            if v is not None:
                return v
            targs = {}
            for p, t in zip((self.inputs[i] for i in self.tensor_pos), tensors):
                targs[p.name] = cg.TensorArg(tuple(t.shape), tuple(t.stride()), t.dtype, t.data_ptr() % 16 == 0)
            rng = {self.inputs[self.number_pos[j]].name: (si, kind) for j, kind, si in rng_key} or None
            ks = cg.generate(self.plan, self.inputs, self.outputs, targs, rng=rng)
            RTC_STATS["generated"] += 1
            v = (load_kernels(ks), ks)
            self._variants[key] = v
            return v

    def __call__(self, *args):
        if _profile.profiling_enabled():
            with _profile.add_markers(self.name):
                return self._call(args)
        return self._call(args)

    def _call(self, args):
        tensors = [args[i] for i in self.tensor_pos]
        dev = tensors[0].device if tensors else None
        if dev is None or dev.type != "cuda":
            return self._run_reference(args)
        outs = [torch.empty(shape, dtype=dt, device=dev) for shape, dt in self._out_specs]
        if self._out_empty or any(t.numel() == 0 for t in tensors):
            return tuple(outs)
        numbers = [args[i] for i in self.number_pos]
        rng_key, states = (), None
        if numbers and any(type(x) is GraphRngInt for x in numbers):
            # Philox arguments drawn inside a hipGraph capture: the kernel reads seed / base from the
            # regions' device RNG states (one pointer per distinct state, after the numbers)
            states, sidx, rk = [], {}, []
            for j, x in enumerate(numbers):
                if type(x) is GraphRngInt:
                    si = sidx.get(id(x.state))
                    if si is None:
                        si = sidx[id(x.state)] = len(states)
                        states.append(x.state)
                    rk.append((j, x.kind, si))
            rng_key = tuple(rk)
        (fns, ks) = self._variant(tensors, rng_key)
        if states:
            launch(ks, fns, tensors, outs, numbers, name=self.name, rng_states=states)
        else:
            launch(ks, fns, tensors, outs, numbers, self._argbuf_t, self._argbuf_ws_t, self.name)
        return tuple(outs)


def arg_buffer_types(n_tensors: int, n_outputs: int, n_numbers: int):
    nwords = n_tensors + max(n_outputs, 1) + n_numbers
    return ctypes.c_uint64 * nwords, ctypes.c_uint64 * (nwords + 1)


def launch(ks: cg.KernelSource, fns: list, tensors: list, outs: list, numbers: list, argbuf_t=None, argbuf_ws_t=None,
           name: str = "hipFusion", rng_states=None) -> None:
    """Launches a generated kernel source (and its extra kernels) with the fusion calling convention:
    one argument block of 64-bit words = input tensor pointers, output pointers (one dummy word when
    there are none), numbers as double bits, the device RNG state pointers of graph-safe Philox
    arguments (``rng_states``), then the workspace pointer when ``ks.ws_bytes``."""
    if rng_states:
        argbuf_t, argbuf_ws_t = arg_buffer_types(len(tensors), len(outs), len(numbers) + len(rng_states))
    elif argbuf_t is None:
        argbuf_t, argbuf_ws_t = arg_buffer_types(len(tensors), len(outs), len(numbers))
    dev = (tensors or outs)[0].device
    buf = argbuf_ws_t() if ks.ws_bytes else argbuf_t()
    k = 0
    for t in tensors:
        buf[k] = t.data_ptr()
        k += 1
    for o in outs:
        buf[k] = o.data_ptr()
        k += 1
    if not outs:
        k += 1
    for x in numbers:
        buf[k] = _double_bits(x)
        k += 1
    for st in rng_states or ():
        buf[k] = st.data_ptr()
        k += 1
    ws = None
    from ..ops._lib import stream_ptr

    if ks.ws_bytes:
        ws = torch.empty(ks.ws_bytes, dtype=torch.uint8, device=dev)  # stream-ordered by the allocator
        buf[k] = ws.data_ptr()
        if ks.counters:
            buf = _with_counters(buf, _counters(ks.counters, dev))

    launches = [(g, b) for _, g, b in ks.pre] + [(ks.grid, ks.block)] + [(g, b) for _, g, b in ks.extra]
    for fn, (grid, block) in zip(fns, launches):
        rc = _lib().lta_rtc_launch(fn, grid[0], grid[1], grid[2], block[0], block[1], block[2], 0, stream_ptr(dev),
                                   ctypes.cast(buf, ctypes.c_void_p), ctypes.sizeof(buf))
        if rc != 0:
            raise RuntimeError(f"{name}: hipModuleLaunchKernel failed with {rc}")
    del ws


_COUNTERS: dict = {}
_CNT_BUF_T: dict = {}


class CaptureCounters:
    """Arrival counters of the column-mode launches captured into one hipGraph: consecutive slices of
    buffers of the graph's own, each zero-filled once by one graph node (every launch leaves its counters
    at zero again, so replays need no re-zeroing) instead of one zero-fill node per launch."""

    CHUNK = 1 << 16

    def __init__(self):
        self.buf = None
        self.used = 0

    def take(self, n: int, dev) -> torch.Tensor:
        n = max(n, 1)
        if self.buf is None or self.buf.device != dev or self.used + n > self.buf.numel():
            self.buf = torch.zeros(max(n, self.CHUNK), dtype=torch.int32, device=dev)
            self.used = 0
        out = self.buf[self.used:self.used + n]
        self.used += (n + 63) // 64 * 64
        return out


_capture_ctx = threading.local()


def set_capture_counters(c) -> None:
    """Installed by HipGraphRunner around a capture (None afterwards)."""
    _capture_ctx.counters = c


def _counters(n: int, dev) -> torch.Tensor:
    """Zeroed uint32 arrival counters of the column-mode kernels: one persistent buffer per (device,
    stream), grown on demand.  Every launch leaves its counters at zero again (the last workgroup of
    each column group resets its own), so kernels ordered on one stream can share it.  Inside a graph
    capture the counters are the graph's own (nothing the graph holds can be shared with or replaced by
    eager launches): slices of the runner's CaptureCounters, else a zero-filled buffer per launch."""
    if torch.cuda.is_current_stream_capturing():
        cc = getattr(_capture_ctx, "counters", None)
        if cc is not None:
            return cc.take(n, dev)
        return torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    buf = _COUNTERS.get(key)
    if buf is None or buf.numel() < n:
        old = buf
        buf = torch.zeros(max(n, 1024), dtype=torch.int32, device=dev)
        if old is not None:  # in-flight launches may still read it: free it behind the stream's work
            old.record_stream(torch.cuda.current_stream(dev))
        _COUNTERS[key] = buf
    return buf


def _with_counters(buf, cnt: torch.Tensor):
    """``buf`` plus one trailing word: the counters pointer (Args ``cnt``)."""
    n = len(buf)
    t = _CNT_BUF_T.get(n)
    if t is None:
        t = _CNT_BUF_T[n] = ctypes.c_uint64 * (n + 1)
    out = t(*buf)
    out[n] = cnt.data_ptr()
    return out


def load_kernels(ks: cg.KernelSource) -> list:
    """Function handles of a kernel source's main kernel and its extra kernels."""
    return ([load_kernel(ks, ks.name + suffix) for suffix, _, _ in ks.pre] + [load_kernel(ks)] +
            [load_kernel(ks, ks.name + suffix) for suffix, _, _ in ks.extra])


def _double_bits(x) -> int:
    import struct

    return struct.unpack("<Q", struct.pack("<d", float(x)))[0]


# -----------------------------------------------------------------------------------------
# Native compile + load (ops/csrc/runtime/rtc.cpp)
# -----------------------------------------------------------------------------------------
_lib_handle = None


def _lib():
    global _lib_handle
    if _lib_handle is None:
        from ..ops import _lib as L

        lib = L.require()
        vp, sz, c_ull = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_ulonglong
        lib.lta_rtc_compile.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(vp),
                                        ctypes.POINTER(sz), ctypes.c_char_p, sz]
        lib.lta_rtc_compile.restype = ctypes.c_int
        lib.lta_rtc_free.argtypes = [vp]
        lib.lta_rtc_free.restype = None
        lib.lta_rtc_load.argtypes = [c_ull, vp, sz, ctypes.c_char_p, ctypes.POINTER(vp)]
        lib.lta_rtc_load.restype = ctypes.c_int
        lib.lta_rtc_launch.argtypes = [vp, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                       ctypes.c_uint, ctypes.c_uint, vp, vp, sz]
        lib.lta_rtc_launch.restype = ctypes.c_int
        _lib_handle = lib
    return _lib_handle


def cache_dir() -> str:
    d = os.environ.get("LTA_CACHE_DIR")
    if not d:
        d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ops", "_build", "rtc_cache")
    os.makedirs(d, exist_ok=True)
    return d


RTC_OPTIONS = "--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast"


# kernel sources generated (one per fusion region and call signature) and hiprtc compiles run (disk
# cache misses) in this process: a symbolic-shape program must not grow them per new size
RTC_STATS = {"generated": 0, "compiled": 0}


def compile_source(ks: cg.KernelSource) -> bytes:
    """HIP source -> gfx950 code object (hiprtc; works without a GPU).  Disk-cached."""
    h = hashlib.sha1((RTC_OPTIONS + ks.src).encode()).hexdigest()
    path = os.path.join(cache_dir(), h + ".co")
    if os.path.exists(path):
        with open(path, "rb") as f:
            return f.read()
    lib = _lib()
    RTC_STATS["compiled"] += 1
    code = ctypes.c_void_p()
    size = ctypes.c_size_t()
    log = ctypes.create_string_buffer(1 << 16)
    rc = lib.lta_rtc_compile(ks.src.encode(), (ks.name + ".hip").encode(), RTC_OPTIONS.encode(), ctypes.byref(code),
                             ctypes.byref(size), log, len(log))
    if rc != 0:
        raise RuntimeError(f"hiprtc failed ({rc}) for {ks.name}:\n{log.value.decode(errors='replace')}\n--- source ---\n{ks.src}")
    data = ctypes.string_at(code, size.value)
    lib.lta_rtc_free(code)
    tmp = path + f".{os.getpid()}.tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)
    return data


def precompile(trace) -> int:
    """Generates and compiles (hiprtc, no GPU needed) the kernel of every hipfuse region of an
    execution trace for dense, 16-byte aligned inputs: an ahead-of-time build check (and disk-cache
    warm-up) that surfaces codegen errors before a GPU run.  Returns the number of regions."""
    from ..core import dtypes as _dt

    fus = fusions(trace)
    for fb in fus:
        f = fb._call_ctx[fb.sym.name]
        targs = {}
        for p in (f.inputs[i] for i in f.tensor_pos):
            shape = tuple(int(x) for x in p.shape)
            targs[p.name] = cg.TensorArg(shape, cg._contig_strides(shape), _dt.to_torch_dtype(p.dtype), True)
        compile_source(cg.generate(f.plan, f.inputs, f.outputs, targs))  # one source: main + pre / extra kernels
    return len(fus)


def load_kernel(ks: cg.KernelSource, name: str | None = None):
    data = compile_source(ks)
    lib = _lib()
    name = name or ks.name
    # one source may define several kernels: the function cache is keyed on (kernel name, source)
    key = int(hashlib.sha1((name + "\0" + ks.src).encode()).hexdigest()[:15], 16)
    fn = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(data, len(data))
    rc = lib.lta_rtc_load(key, buf, len(data), name.encode(), ctypes.byref(fn))
    if rc != 0:
        raise RuntimeError(f"loading {name} failed with HIP error {rc}")
    return fn.value


# -----------------------------------------------------------------------------------------
# Fusion pass
# -----------------------------------------------------------------------------------------
def _connected(plan_names: set, group_inputs: set, b: BoundSymbol) -> bool:
    for a in b.flat_proxy_args:
        if a.name in plan_names or a.name in group_inputs:
            return True
    return False


def _external_view(names: set, b: BoundSymbol) -> bool:
    """Views (broadcasts, reshapes, slices, ...) and gathers / concatenations of values produced
    outside the open region are free to join it (e.g. a position-embedding lookup joins the region
    that adds it to the token embeddings)."""
    return (b.sym.id in cg.VIEWS or b.sym.id in cg.GATHERS) and not any(a.name in names for a in b.flat_proxy_args)


_LAZY: set = set()  # names of lazily re-materialised casts of the trace being partitioned


def _is_widening_convert(b: BoundSymbol) -> bool:
    if b.sym.id != PrimIDs.CONVERT_ELEMENT_TYPE or not isinstance(b.args[0], TensorProxy):
        return False
    return b.output.dtype.itemsize > b.args[0].dtype.itemsize


def _schedule_segment(seg: list, used_outside: set | None = None) -> list:
    """Dataflow partition of a side-effect-free segment -> list of bsyms and groups (lists).

    Widening casts (bf16 -> fp32, ...) are *lazy*: they are never scheduled on their own but
    re-materialised inside every region that consumes them (or once, standalone, before a
    non-fusible consumer), so a region never writes an upcast copy of a tensor to HBM just
    because a later region reads it in fp32.
    """
    used_outside = used_outside or set()
    n = len(seg)
    prod: dict[str, int] = {}
    for i, b in enumerate(seg):
        for o in b.flat_proxy_outs:
            prod[o.name] = i
    deps = [set() for _ in range(n)]
    users = [[] for _ in range(n)]
    for i, b in enumerate(seg):
        for a in b.flat_proxy_args:
            j = prod.get(a.name)
            if j is not None and j != i and j not in deps[i]:
                deps[i].add(j)
                users[j].append(i)
    fusible = [_fusible_leaf(b) for b in seg]
    lazy = [False] * n
    for i, b in enumerate(seg):
        if fusible[i] and _is_widening_convert(b) and not any(o.name in used_outside for o in b.flat_proxy_outs):
            lazy[i] = True
    for i in range(n):
        if lazy[i] and any(lazy[d] for d in deps[i]):
            lazy[i] = False
    lazy_deps = [{d for d in deps[i] if lazy[d]} for i in range(n)]
    materialized: set[int] = set()  # lazy nodes already emitted standalone
    for i in range(n):
        if lazy[i]:
            _LAZY.update(o.name for o in seg[i].flat_proxy_outs)
    indeg = [len(d) for d in deps]
    ready: list = []
    items: list = []
    plan = None
    group: list = []
    in_group: set[int] = set()
    names: set = set()
    ins: set = set()

    def done(i):
        for u in users[i]:
            indeg[u] -= 1
            if indeg[u] == 0:
                if lazy[u]:
                    done(u)  # available on demand: its consumers may become ready
                else:
                    heapq.heappush(ready, u)

    for i in [i for i in range(n) if indeg[i] == 0]:
        if lazy[i]:
            done(i)
        else:
            heapq.heappush(ready, i)

    def close():
        nonlocal plan, group, names, ins, in_group
        if group:
            items.append((plan, group))
        plan, group, names, ins, in_group = None, [], set(), set(), set()

    def add_to_group(idxs):
        nonlocal names, ins
        for j in idxs:
            group.append(seg[j])
            in_group.add(j)
            names |= {o.name for o in seg[j].flat_proxy_outs}
            ins |= {a.name for a in seg[j].flat_proxy_args if isinstance(a, TensorProxy)}

    def try_admit(i) -> bool:
        extra = [d for d in sorted(lazy_deps[i]) if d not in in_group and d not in materialized]
        trial = plan.copy()
        for j in extra + [i]:
            if not trial.try_add(seg[j]):
                return False
        if trial.has_pending():
            return False
        plan.__dict__.update(trial.__dict__)
        add_to_group(extra + [i])
        return True

    from ..common import get_compile_option

    fusion_type = get_compile_option(
        "fusion_type", "hipfuse partitioner: 'dataflow' (default: any ready, connected bound symbol may join the "
        "open region) or 'consecutive' (only the next bound symbol in program order)", "dataflow")
    if fusion_type not in ("dataflow", "consecutive"):
        raise ValueError(f"fusion_type must be 'dataflow' or 'consecutive', got {fusion_type!r}")
    consecutive = fusion_type == "consecutive"

    def feeds_region(i, depth=6) -> bool:
        """A source (no tensor inputs: an RNG draw, a ``full``) joins the open region when a fusible
        consumer within a few hops also reads the region's values (e.g. the dropout mask of a
        dropout backward whose gradient the region produces)."""
        if any(isinstance(a, TensorProxy) for a in seg[i].flat_proxy_args):
            return False
        frontier, seen = [i], {i}
        for _ in range(depth):
            nxt = []
            for j in frontier:
                for u in users[j]:
                    if u in seen or not fusible[u]:
                        continue
                    seen.add(u)
                    if any(a.name in names for a in seg[u].flat_proxy_args):
                        return True
                    nxt.append(u)
            frontier = nxt
        return False

    while ready:
        pick = None
        if plan is not None:
            for i in (sorted(ready)[:1] if consecutive else sorted(ready)):
                if fusible[i] and (_connected(names, ins, seg[i]) or _external_view(names, seg[i]) or
                                   any(d in in_group or _connected(names, ins, seg[d]) for d in lazy_deps[i]) or
                                   (not consecutive and feeds_region(i))) \
                        and try_admit(i):
                    pick = i
                    break
        if pick is not None:
            ready.remove(pick)
            heapq.heapify(ready)
            done(pick)
            continue
        close()
        i = heapq.heappop(ready)
        b = seg[i]
        started = False
        if fusible[i]:
            plan = cg.Plan()
            if try_admit(i):
                started = True
            else:
                plan = None
        if not started:
            for d in sorted(lazy_deps[i]):
                if d not in materialized:
                    materialized.add(d)
                    items.append(seg[d])
            items.append(b)
        done(i)
    close()
    return items


def _fusion_pass(trace):
    flat: list[BoundSymbol] = []
    for b in trace.bound_symbols:
        flat.extend(_flatten(b))
    # segment boundaries and the names each segment must export to the rest of the trace
    segments: list = []
    seg: list = []
    for b in flat:
        if _is_barrier(b) or not (b.flat_proxy_outs or b.flat_proxy_args):
            if seg:
                segments.append(seg)
                seg = []
            segments.append(b)
        else:
            seg.append(b)
    if seg:
        segments.append(seg)
    _LAZY.clear()
    uses_by_seg: list[set] = []
    for s_ in segments:
        bs = s_ if isinstance(s_, list) else [s_]
        uses_by_seg.append({a.name for b in bs for a in b.flat_proxy_args})
    items: list = []
    for k, s_ in enumerate(segments):
        if not isinstance(s_, list):
            items.append(s_)
            continue
        outside = set()
        for j, u in enumerate(uses_by_seg):
            if j != k:
                outside |= u
        items.extend(_schedule_segment(s_, outside))

    from ..common import get_compile_option

    remat_names = {}
    if get_compile_option("fusion_type", "hipfuse partitioner mode", "dataflow") != "consecutive" and \
            get_compile_option("hipfuse_rematerialize", "recompute cheap producer cones of values passed between "
                               "hipfuse regions instead of materialising them (default True)", True):
        remat_names = _rematerialize_between_regions(items)
    lazy_names = set(_LAZY)
    # consumers outside each group decide region outputs
    use_count: dict[str, list] = {}
    for idx, it in enumerate(items):
        bs = it[1] if isinstance(it, tuple) else [it]
        inside = remat_names.get(idx, ())  # recomputed here: these reads are internal to the region
        for b in bs:
            for a in b.flat_proxy_args:
                if a.name not in inside:
                    use_count.setdefault(a.name, []).append(idx)
    new_bsyms: list = []
    for idx, it in enumerate(items):
        if not isinstance(it, tuple):
            new_bsyms.append(it)
            continue
        plan, group = it
        # views of external values: never materialise them as region outputs
        pre = []
        internal_names = set()
        for b in group:
            if not (b.sym.id in cg.VIEWS and not any(a.name in internal_names for a in b.flat_proxy_args)):
                internal_names |= {o.name for o in b.flat_proxy_outs}
        used_inside = {a.name for b in group for a in b.flat_proxy_args}
        original = list(group)

        def is_ext_view(b):
            return b.sym.id in cg.VIEWS and not any(a.name in internal_names for a in b.flat_proxy_args)

        # ext views needed outside the region are emitted standalone before it, together with the
        # ext views they are built from (closed under ancestry, kept in group order)
        need: set[str] = set()
        for b in group:
            if is_ext_view(b):
                o = b.flat_proxy_outs[0].name
                if any(u != idx for u in use_count.get(o, [])) and o not in remat_names.get(idx, ()):
                    need.add(o)
        for b in reversed(group):
            if is_ext_view(b) and b.flat_proxy_outs[0].name in need:
                need |= {a.name for a in b.flat_proxy_args}
        pre = [b for b in group if is_ext_view(b) and b.flat_proxy_outs[0].name in need]
        keep = [b for b in group if not (is_ext_view(b) and b.flat_proxy_outs[0].name not in used_inside)]
        # trailing view chains of region values ending in a transpose (autodiff's wgrad operand
        # dY^T of an elementwise producer): the region stores the base value and the views run
        # standalone after it (zero-copy; the GEMMs read transposed operands in place) instead of the
        # region storing a transposed copy with strided 2-byte stores (Gemma's GeGLU backward: 2.4 ms)
        post = _trailing_views(keep, internal_names, lazy_names | set(remat_names.get(idx, ())))
        if post:
            post_ids = {id(b) for b in post}
            keep = [b for b in keep if id(b) not in post_ids]
            for b in post:
                for a_ in b.flat_proxy_args:
                    use_count.setdefault(a_.name, []).append(-1 - idx)
        if len(keep) != len(group):
            plan = _replan(keep)
            if plan is None:
                new_bsyms.extend(original)
                continue
            group = keep
        ncompute = sum(1 for b in group if cg.is_compute(b))
        if ncompute < 2 or not ex.get_fuel():
            new_bsyms.extend(original)
            continue
        new_bsyms.extend(pre)
        post_after = post
        pre_names = {o.name for b in pre for o in b.flat_proxy_outs}
        produced = []
        pset = set()
        for b in group:
            for o in b.flat_proxy_outs:
                if o.name in pset:
                    continue
                produced.append(o)
                pset.add(o.name)
        outputs = [o for o in produced if o.name not in pre_names and o.name not in lazy_names
                   and o.name not in remat_names.get(idx, ())
                   and any(u != idx for u in use_count.get(o.name, []))]
        seen = set()
        inputs = []
        for b in group:
            for a in b.flat_proxy_args:
                if a.name not in pset and a.name not in seen:
                    seen.add(a.name)
                    inputs.append(a)
        if not outputs:
            continue
        name = f"hipFusion{next(_counter)}"
        fn = HipFusion(name, plan, inputs, outputs, list(group))
        sym = Symbol(name, meta=None, is_prim=True, executor=ex, is_fusion=True)
        nb = BoundSymbol(sym, args=tuple(inputs), kwargs={}, output=tuple(outputs), subsymbols=list(group),
                         _call_ctx={name: fn})
        new_bsyms.append(nb)
        new_bsyms.extend(post_after)
    new = from_trace(trace)
    new.bound_symbols = new_bsyms
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance("Fusion (hipfuse)"))
    return new


def _trailing_views(group: list, internal_names: set, unstorable: set = frozenset()) -> list:
    """View ops at the end of a region's dataflow (outputs read by no other op of the region) that
    form chains ending in a transpose of a region value; [] when there is no transpose among them, or
    when a chain starts from a value the region cannot hand out (``unstorable``: lazily re-materialised
    casts, values recomputed from other regions)."""
    moved: list = []
    mids: set = set()
    remaining = list(group)
    while True:
        used = {a.name for b in remaining for a in b.flat_proxy_args}
        cand = [b for b in remaining if b.sym.id in cg.VIEWS and b.flat_proxy_outs
                and all(o.name not in used for o in b.flat_proxy_outs)
                and any(a.name in internal_names for a in b.flat_proxy_args)]
        if not cand:
            break
        ids = {id(b) for b in cand}
        moved.extend(cand)
        mids |= ids
        remaining = [b for b in remaining if id(b) not in ids]
    if not any(b.sym.id == PrimIDs.TRANSPOSE for b in moved):
        return []
    moved_outs = {o.name for b in moved for o in b.flat_proxy_outs}
    if any(a.name in unstorable for b in moved for a in b.flat_proxy_args if a.name not in moved_outs):
        return []
    if not any(cg.is_compute(b) for b in remaining):
        return []
    return [b for b in group if id(b) in mids]  # program order


def _tensor_bytes(p) -> int:
    n = p.numel
    return int(n) * p.dtype.itemsize if isinstance(n, int) else 0


def _rematerialize_between_regions(items: list) -> dict:
    """Fusion-region rematerialisation (reference: ``thunder/core/rematerialization.py:239-407``,
    the min-cut between adjacent nvFuser regions).  When a region reads a value X that an earlier
    region produces only for it, and X's producer cone inside the earlier region (elementwise /
    view / gather prims, no reduction) reads fewer bytes than X's HBM round trip (write + read),
    the cone is recomputed inside the consumer and X is never materialised.  Returns, per item
    index, the names the consumer recomputes (they must not become its outputs: their original
    region still defines them for any other user)."""
    remat: dict[int, set] = {}
    group_pos = [i for i, it in enumerate(items) if isinstance(it, tuple)]
    if len(group_pos) < 2:
        return remat
    producer_item: dict[str, int] = {}
    uses: dict[str, set] = {}
    for idx, it in enumerate(items):
        bs = it[1] if isinstance(it, tuple) else [it]
        for b in bs:
            for a in b.flat_proxy_args:
                uses.setdefault(a.name, set()).add(idx)
            for o in b.flat_proxy_outs:
                producer_item.setdefault(o.name, idx)
    cheap = cg.ELEMENTWISE | cg.VIEWS | cg.GATHERS | {PrimIDs.FULL, PrimIDs.UNIFORM_PHILOX}
    for j in group_pos:
        for _ in range(8):  # a few rounds: a recomputed cone can expose the next candidate
            plan2, g2 = items[j]
            made = {o.name for b in g2 for o in b.flat_proxy_outs}
            ext, ext_names = [], set()
            for b in g2:
                for a in b.flat_proxy_args:
                    if isinstance(a, TensorProxy) and a.name not in made and a.name not in ext_names:
                        ext.append(a)
                        ext_names.add(a.name)
            done = False
            for x in ext:
                i = producer_item.get(x.name)
                if i is None or i >= j or not isinstance(items[i], tuple) or uses.get(x.name, set()) - {i, j}:
                    continue
                g1 = items[i][1]
                prod = {o.name: b for b in g1 for o in b.flat_proxy_outs}
                cone, stack, seen = [], [x.name], set()
                ok = True
                while stack and ok:
                    n = stack.pop()
                    if n in made:  # already computed inside the consumer (an earlier recomputed cone)
                        continue
                    b = prod.get(n)
                    if b is None or id(b) in seen:
                        continue
                    seen.add(id(b))
                    if b.sym.id not in cheap:
                        ok = False
                        break
                    cone.append(b)
                    stack.extend(a.name for a in b.flat_proxy_args if isinstance(a, TensorProxy))
                if not ok or not cone:
                    continue
                cone = [b for b in g1 if id(b) in seen]  # program order
                cone_made = {o.name for b in cone for o in b.flat_proxy_outs}
                reads = {a.name: a for b in cone for a in b.flat_proxy_args
                         if isinstance(a, TensorProxy) and a.name not in cone_made}
                extra = sum(_tensor_bytes(a) for n, a in reads.items() if n not in ext_names)
                if extra >= 2 * _tensor_bytes(x):
                    continue
                merged = _topo_order(cone + list(g2))
                trial = cg.Plan()
                if not all(trial.try_add(b) for b in merged) or trial.has_pending():
                    continue
                items[j] = (trial, merged)
                remat.setdefault(j, set()).update(cone_made)
                uses[x.name].discard(j)
                for n in reads:
                    uses.setdefault(n, set()).add(j)
                done = True
                break
            if not done:
                break
    return remat


def _topo_order(bsyms: list) -> list:
    """``bsyms`` in a dependency-respecting order, as close to the given order as possible (a
    recomputed cone may read values an earlier recomputed cone defines inside the consumer)."""
    prod = {}
    for k, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            prod.setdefault(o.name, k)
    out, placed = [], set()

    def place(k, stack=()):
        if k in placed:
            return
        for a in bsyms[k].flat_proxy_args:
            d = prod.get(a.name)
            if d is not None and d != k and d not in stack:
                place(d, stack + (k,))
        placed.add(k)
        out.append(bsyms[k])

    for k in range(len(bsyms)):
        place(k)
    return out


def _replan(group):
    plan = cg.Plan()
    for b in group:
        if not plan.try_add(b):
            return None
    return plan


ex.fusion_pass = _fusion_pass


def fusions(trace) -> list:
    """The hipFusion bound symbols of an execution trace."""
    return [b for b in trace.bound_symbols if b.sym.is_fusion and b.sym.executor is ex]
