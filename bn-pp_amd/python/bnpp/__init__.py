"""ctypes binding of the bn-pp MI355X engine (include/bnpp.h).

This is plumbing for tests and bench.py: every call goes straight to
bn-pp_amd/lib/libbnpp.so.  There is no Python or CPU fallback — a missing
library raises ImportError and a missing GPU raises BnppError(NO_DEVICE).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Iterable, List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libbnpp.so"))
if os.environ.get("BNPP_LIB"):          # A/B of alternative builds (experiments only)
    LIB_PATH = os.environ["BNPP_LIB"]

if not os.path.exists(LIB_PATH):
    raise ImportError("libbnpp.so not built (%s); run `make -C bn-pp_amd` or __graft_entry__.build()" % LIB_PATH)

# One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.  When it
# is installed, load it first so libbnpp binds to that same runtime (with two
# runtimes in one process, whichever initialises second sees no device).
# BNPP_NO_TORCH=1 leaves PyTorch out of a process that does not use it: libbnpp
# then binds to ROCm's runtime.  That is also the way to run under
# HIP_ENABLE_DEFERRED_LOADING=0, where `import torch` itself segfaults on this
# image (PyTorch 2.10+rocm7.0, inside `from torch._C import *`).
if os.environ.get("BNPP_NO_TORCH") != "1":
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
_lib = C.CDLL(LIB_PATH)

OK, ERR_INVALID, ERR_NO_DEVICE, ERR_OOM, ERR_HIP, ERR_IO, ERR_UNSUPPORTED = 0, -1, -2, -3, -4, -5, -6
F64, F32 = 0, 1
ORDER_GIVEN, MIN_FILL, WEIGHTED_MIN_FILL, MIN_DEGREE = 0, 1, 2, 3
HEURISTICS = {"given": ORDER_GIVEN, "mf": MIN_FILL, "wmf": WEIGHTED_MIN_FILL, "md": MIN_DEGREE}

_P = C.c_void_p
_I = C.c_int
_IP = C.POINTER(C.c_int)
_DP = C.POINTER(C.c_double)
_LP = C.POINTER(C.c_int64)
# bnpp_collective_fn (include/bnpp.h): (user, op, send, recv, bytes, stream) -> 0 on success
COLLECTIVE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)
COLL_ALLGATHER, COLL_ALLTOALL = 0, 1

_SIGS = {
    "bnpp_strerror": (C.c_char_p, [_I]),
    "bnpp_last_error": (C.c_char_p, []),
    "bnpp_version": (_I, []),
    "bnpp_last_timing": (_I, [_DP, _I]),
    "bnpp_device_count": (_I, [_IP]),
    "bnpp_ctx_create": (_I, [_I, C.POINTER(_P)]),
    "bnpp_ctx_destroy": (_I, [_P]),
    "bnpp_ctx_stream": (_I, [_P, C.POINTER(_P)]),
    "bnpp_ctx_trim": (_I, [_P]),
    "bnpp_malloc": (_I, [_P, C.c_size_t, C.POINTER(_P)]),
    "bnpp_free": (_I, [_P, _P]),
    "bnpp_memcpy_h2d": (_I, [_P, _P, _P, C.c_size_t]),
    "bnpp_memcpy_d2h": (_I, [_P, _P, _P, C.c_size_t]),
    "bnpp_synchronize": (_I, [_P, _P]),
    "bnpp_out_scope": (_I, [_I, _IP, C.POINTER(_IP), _I, _I, _IP, _IP]),
    "bnpp_bucket_eliminate": (_I, [_P, _P, _I, _I, _IP, _I, C.POINTER(_P), _IP, C.POINTER(_IP), _I, _P, _I, _IP, _P]),
    "bnpp_product": (_I, [_P, _P, _I, _I, _IP, _P, _I, _IP, _P, _I, _IP, _P, _I, _IP, _P]),
    "bnpp_divide": (_I, [_P, _P, _I, _I, _IP, _P, _I, _IP, _P, _I, _IP, _P, _I, _IP, _P]),
    "bnpp_sum_out": (_I, [_P, _P, _I, _I, _IP, _P, _I, _IP, _I, _P, _I, _IP, _P]),
    "bnpp_condition": (_I, [_P, _P, _I, _I, _IP, _P, _I, _IP, _I, _IP, _IP, _P, _P]),
    "bnpp_model_load_uai": (_I, [C.c_char_p, C.POINTER(_P)]),
    "bnpp_model_from_arrays": (_I, [_I, _I, _IP, _I, _IP, _IP, _DP, C.POINTER(_P)]),
    "bnpp_model_free": (_I, [_P]),
    "bnpp_model_info": (_I, [_P, _IP, _IP, _IP]),
    "bnpp_model_cards": (_I, [_P, _IP]),
    "bnpp_evidence_load": (_I, [C.c_char_p, _I, _IP, _IP, _IP]),
    "bnpp_ordering": (_I, [_P, _I, _IP, _IP, _I, _IP, _I, _IP, _IP]),
    "bnpp_partition": (_I, [_P, _P, _I, _IP, _IP, _I, _IP, _I, _I, _DP, _DP, _DP]),
    "bnpp_marginals": (_I, [_P, _P, _I, _IP, _IP, _I, _I, _IP, _I, _DP, _DP]),
    "bnpp_sum_product": (_I, [_P, _P, _I, C.c_double, _DP, _IP, _DP]),
    "bnpp_marginals_tree": (_I, [_P, _P, _I, _IP, _IP, _I, _IP, _I, _I, _IP, _I, _DP, _DP]),
    "bnpp_marginals_tree_part": (_I, [_P, _P, _I, _IP, _IP, _I, _IP, _I, _I, _IP, _I, _I, _I, _DP, _IP, _DP]),
    "bnpp_plan_tree_part": (_I, [_P, _I, _IP, _IP, _I, _IP, _I, _I, _I, _I, _IP, _DP, _I]),
    "bnpp_marginals_tree_sliced": (_I, [_P, _P, _I, _IP, _IP, _I, _IP, _I, _I, _IP, _I, _I, COLLECTIVE_FN, _P,
                                        C.c_double, _I, _DP, _LP, _DP]),
    "bnpp_collective_loopback": (_I, [_P, _I, _P, _P, C.c_int64, _P]),
    "bnpp_plan_tree_sliced": (_I, [_P, _I, _IP, _IP, _I, _IP, _I, _I, _I, _I, _IP, _DP, _I]),
    "bnpp_variable_elimination": (_I, [_P, _P, _I, _IP, _I, _I, _I, _IP, _IP, C.c_int64, C.POINTER(C.c_int64), _DP,
                                       C.POINTER(C.c_int64)]),
    "bnpp_plan_stats": (_I, [_P, _I, _I, _IP, _IP, _I, _IP, _I, _I, _DP, _I]),
    "bnpp_job_create": (_I, [_P, _P, _I, _I, _IP, _IP, _I, _IP, _I, _I, _IP, _I, C.POINTER(_P)]),
    "bnpp_job_stats": (_I, [_P, _DP, _I]),
    "bnpp_job_launch": (_I, [_P, _P]),
    "bnpp_job_results": (_I, [_P, _P, _DP]),
    "bnpp_job_free": (_I, [_P]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = sorted(_SIGS)

# The signature table above is for this ABI version (include/bnpp.h
# BNPP_VERSION); a library of another version would take shifted arguments.
ABI_VERSION = 202
if _lib.bnpp_version() != ABI_VERSION:
    raise ImportError("libbnpp.so ABI version %d, this binding expects %d (%s)"
                      % (_lib.bnpp_version(), ABI_VERSION, LIB_PATH))


class BnppError(RuntimeError):
    def __init__(self, status: int, where: str):
        self.status = status
        super().__init__("%s: %s (%s)" % (where, _lib.bnpp_strerror(status).decode(), _lib.bnpp_last_error().decode()))


def _check(rc: int, where: str) -> None:
    if rc != OK:
        raise BnppError(rc, where)


def _ints(xs: Iterable[int]):
    xs = list(xs)
    return (C.c_int * max(len(xs), 1))(*xs)


def _dbls(xs: Iterable[float]):
    xs = list(xs)
    return (C.c_double * max(len(xs), 1))(*xs)


TIMING_PHASES = ("plan_ms", "upload_ms", "program_ms", "launch_ms", "run_fetch_ms", "free_ms", "total_ms",
                 "arena_reused", "arena_alloc_ms")


def last_timing() -> Dict[str, float]:
    """Phase split of this thread's last partition / marginals call (bnpp_last_timing)."""
    out = (C.c_double * len(TIMING_PHASES))()
    _check(_lib.bnpp_last_timing(out, len(TIMING_PHASES)), "bnpp_last_timing")
    return dict(zip(TIMING_PHASES, list(out)))


def device_count() -> int:
    n = C.c_int(0)
    _check(_lib.bnpp_device_count(C.byref(n)), "bnpp_device_count")
    return n.value


class Context:
    """One device context (bnpp_ctx_create).  Fails with NO_DEVICE without a GPU."""

    def __init__(self, device: int = 0):
        self._h = _P()
        _check(_lib.bnpp_ctx_create(device, C.byref(self._h)), "bnpp_ctx_create")
        self.device = device

    @property
    def handle(self):
        return self._h

    def trim(self) -> None:
        """Release the device memory kept between calls (cached arena, buffers)."""
        _check(_lib.bnpp_ctx_trim(self.handle), "bnpp_ctx_trim")

    def stream(self) -> int:
        s = _P()
        _check(_lib.bnpp_ctx_stream(self._h, C.byref(s)), "bnpp_ctx_stream")
        return s.value or 0

    def synchronize(self, stream: Optional[int] = None) -> None:
        _check(_lib.bnpp_synchronize(self._h, _P(stream) if stream else None), "bnpp_synchronize")

    def close(self) -> None:
        if self._h:
            _lib.bnpp_ctx_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Model:
    """A UAI model held by the engine (host memory)."""

    def __init__(self, handle):
        self._h = handle
        ib, nv, nf = C.c_int(), C.c_int(), C.c_int()
        _check(_lib.bnpp_model_info(self._h, C.byref(ib), C.byref(nv), C.byref(nf)), "bnpp_model_info")
        self.is_bayes, self.n_vars, self.n_factors = bool(ib.value), nv.value, nf.value
        cards = (C.c_int * max(nv.value, 1))()
        _check(_lib.bnpp_model_cards(self._h, cards), "bnpp_model_cards")
        self.cards = list(cards[: nv.value])

    @classmethod
    def load(cls, path: str) -> "Model":
        h = _P()
        _check(_lib.bnpp_model_load_uai(path.encode(), C.byref(h)), "bnpp_model_load_uai")
        return cls(h)

    @classmethod
    def from_dict(cls, m: dict) -> "Model":
        widths = [len(s) for s in m["scopes"]]
        scopes = [v for s in m["scopes"] for v in s]
        values = [x for vals in m["values"] for x in vals]
        h = _P()
        _check(_lib.bnpp_model_from_arrays(1 if m.get("type") == "BAYES" else 0, len(m["cards"]), _ints(m["cards"]),
                                           len(widths), _ints(widths), _ints(scopes), _dbls(values), C.byref(h)),
               "bnpp_model_from_arrays")
        return cls(h)

    @classmethod
    def from_arrays(cls, cards: Sequence[int], scopes: Sequence[Sequence[int]], values, is_bayes: bool = False
                    ) -> "Model":
        """A model from one flat float64 array of every factor's table in
        order (numpy, C-contiguous, passed by pointer: no per-entry Python
        objects, so tables of billions of entries load in seconds)."""
        import numpy as np
        vals = np.ascontiguousarray(values, dtype=np.float64).reshape(-1)
        widths = [len(s) for s in scopes]
        flat = [v for s in scopes for v in s]
        h = _P()
        _check(_lib.bnpp_model_from_arrays(1 if is_bayes else 0, len(cards), _ints(cards), len(widths), _ints(widths),
                                           _ints(flat), vals.ctypes.data_as(_DP), C.byref(h)),
               "bnpp_model_from_arrays")
        return cls(h)

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            if self._h:
                _lib.bnpp_model_free(self._h)
                self._h = _P()
        except Exception:
            pass


def _ev(evidence: Optional[Dict[int, int]]):
    evidence = evidence or {}
    ks = sorted(evidence)
    return len(ks), _ints(ks), _ints([evidence[k] for k in ks])


def load_evidence(path: str) -> Dict[int, int]:
    cap = 1 << 16
    n = C.c_int()
    vs, xs = (C.c_int * cap)(), (C.c_int * cap)()
    _check(_lib.bnpp_evidence_load(path.encode(), cap, C.byref(n), vs, xs), "bnpp_evidence_load")
    return {vs[i]: xs[i] for i in range(n.value)}


def ordering(model: Model, evidence=None, heuristic: str = "mf", variables: Optional[Sequence[int]] = None):
    n, ev_v, ev_x = _ev(evidence)
    out = (C.c_int * max(model.n_vars, 1))()
    w = C.c_int()
    if variables is None:
        _check(_lib.bnpp_ordering(model.handle, n, ev_v, ev_x, 0, None, HEURISTICS[heuristic], out, C.byref(w)),
               "bnpp_ordering")
        cnt = model.n_vars - len(evidence or {})
    else:
        variables = list(variables)
        _check(_lib.bnpp_ordering(model.handle, n, ev_v, ev_x, len(variables), _ints(variables), HEURISTICS[heuristic],
                                  out, C.byref(w)), "bnpp_ordering")
        cnt = len(variables)
    return list(out[:cnt]), w.value


def out_scope(scopes: Sequence[Sequence[int]], elim: int = -1) -> List[int]:
    arrs = [_ints(s) for s in scopes]
    ptrs = (_IP * max(len(arrs), 1))(*[C.cast(a, _IP) for a in arrs])
    nd = _ints([len(s) for s in scopes])
    cap = sum(len(s) for s in scopes) + 1
    out = (C.c_int * cap)()
    n = C.c_int()
    _check(_lib.bnpp_out_scope(len(scopes), nd, ptrs, elim, cap, C.byref(n), out), "bnpp_out_scope")
    return list(out[: n.value])


def plan_stats(model: Model, kind: int = 0, evidence=None, heuristic: str = "mf", dtype: int = F64,
               order: Optional[Sequence[int]] = None) -> List[float]:
    n, ev_v, ev_x = _ev(evidence)
    st = (C.c_double * 8)()
    oa = _ints(order) if order is not None else None
    h = ORDER_GIVEN if order is not None else HEURISTICS[heuristic]
    _check(_lib.bnpp_plan_stats(model.handle, kind, n, ev_v, ev_x, h, oa, len(order) if order is not None else 0,
                                dtype, st, 8), "bnpp_plan_stats")
    return list(st)


def partition(ctx: Context, model: Model, evidence=None, heuristic: str = "mf", dtype: int = F64,
              order: Optional[Sequence[int]] = None):
    """BN::partition (model.cpp:250-301) -> (log10 Z, Z, uptime_ms)."""
    n, ev_v, ev_x = _ev(evidence)
    lz, z, up = C.c_double(), C.c_double(), C.c_double()
    if order is not None:
        order = list(order)
        _check(_lib.bnpp_partition(ctx.handle, model.handle, n, ev_v, ev_x, ORDER_GIVEN, _ints(order), len(order), dtype,
                                   C.byref(lz), C.byref(z), C.byref(up)), "bnpp_partition")
    else:
        _check(_lib.bnpp_partition(ctx.handle, model.handle, n, ev_v, ev_x, HEURISTICS[heuristic], None, 0, dtype,
                                   C.byref(lz), C.byref(z), C.byref(up)), "bnpp_partition")
    return lz.value, z.value, up.value


def marginals(ctx: Context, model: Model, evidence=None, heuristic: str = "mf", dtype: int = F64,
              targets: Optional[Sequence[int]] = None):
    """BN::marginals (model.cpp:303-346) -> ({var: [p_0..p_k-1]}, uptime_ms)."""
    n, ev_v, ev_x = _ev(evidence)
    tg = list(range(model.n_vars)) if targets is None else list(targets)
    total = sum(model.cards[t] for t in tg)
    out = (C.c_double * max(total, 1))()
    up = C.c_double()
    _check(_lib.bnpp_marginals(ctx.handle, model.handle, n, ev_v, ev_x, HEURISTICS[heuristic], len(tg), _ints(tg),
                               dtype, out, C.byref(up)), "bnpp_marginals")
    res, o = {}, 0
    for t in tg:
        res[t] = list(out[o:o + model.cards[t]])
        o += model.cards[t]
    return res, up.value


def sum_product(ctx: Context, model: Model, max_iter: int = 10000, eps: float = 0.001):
    """BN::marginals with options["sum-product"] (model.cpp:313-317): loopy BP
    on the device (bnpp_sum_product) -> ({var: [p_0..p_k-1]}, iterations, uptime_ms).
    Evidence is not used on this path, as in the reference."""
    out = (C.c_double * max(sum(model.cards), 1))()
    it, up = C.c_int(), C.c_double()
    _check(_lib.bnpp_sum_product(ctx.handle, model.handle, max_iter, eps, out, C.byref(it), C.byref(up)),
           "bnpp_sum_product")
    res, o = {}, 0
    for t in range(model.n_vars):
        res[t] = list(out[o:o + model.cards[t]])
        o += model.cards[t]
    return res, it.value, up.value


def marginals_tree(ctx: Context, model: Model, evidence=None, heuristic: str = "mf", dtype: int = F64,
                   targets: Optional[Sequence[int]] = None, order: Optional[Sequence[int]] = None,
                   part: int = 0, n_parts: int = 1):
    """All marginals from one two-pass bucket tree (bnpp_marginals_tree) ->
    ({var: [p_0..p_k-1]}, uptime_ms).  Same output as marginals(), to rounding.
    part / n_parts (bnpp_marginals_tree_part): only the targets this part owns."""
    n, ev_v, ev_x = _ev(evidence)
    tg = list(range(model.n_vars)) if targets is None else list(targets)
    total = sum(model.cards[t] for t in tg)
    out = (C.c_double * max(total, 1))()
    owned = (C.c_int * max(len(tg), 1))()
    up = C.c_double()
    oa = _ints(list(order)) if order is not None else None
    h = ORDER_GIVEN if order is not None else HEURISTICS[heuristic]
    _check(_lib.bnpp_marginals_tree_part(ctx.handle, model.handle, n, ev_v, ev_x, h, oa,
                                         len(order) if order is not None else 0, len(tg), _ints(tg), part, n_parts,
                                         dtype, out, owned, C.byref(up)), "bnpp_marginals_tree_part")
    res, o = {}, 0
    for i, t in enumerate(tg):
        if owned[i]:
            res[t] = list(out[o:o + model.cards[t]])
        o += model.cards[t]
    return res, up.value


def plan_tree_part(model: Model, part: int, n_parts: int, evidence=None, heuristic: str = "mf", dtype: int = F64,
                   order: Optional[Sequence[int]] = None):
    """Host-only plan of one part of the bucket-tree marginals ->
    (owned variable ids, stats list as Job)."""
    n, ev_v, ev_x = _ev(evidence)
    owned = (C.c_int * max(model.n_vars, 1))()
    st = (C.c_double * 8)()
    oa = _ints(list(order)) if order is not None else None
    h = ORDER_GIVEN if order is not None else HEURISTICS[heuristic]
    _check(_lib.bnpp_plan_tree_part(model.handle, n, ev_v, ev_x, h, oa, len(order) if order is not None else 0,
                                    part, n_parts, dtype, owned, st, 8), "bnpp_plan_tree_part")
    return [v for v in range(model.n_vars) if owned[v]], list(st)


NO_EXP = -(1 << 40)       # out_exp2 of an all-zero share (include/bnpp.h)


def marginals_tree_sliced(ctx: Context, model: Model, rank: int, n_ranks: int, collective, evidence=None,
                          heuristic: str = "mf", dtype: int = F32, targets: Optional[Sequence[int]] = None,
                          order: Optional[Sequence[int]] = None, budget_gb: float = 0.0):
    """This rank's share of the message-sliced bucket-tree marginals
    (bnpp_marginals_tree_sliced) -> ({var: mantissas}, {var: exp2}, uptime_ms);
    the marginal of v is the normalised sum over ranks of mantissas * 2^exp2
    (bnpp.dist.sliced_tree_marginals).  collective: "loopback" (one GPU, a
    world of identical ranks: timing only; "loopback-nocopy": no bytes move)
    or callable(op, send, recv, nbytes,
    stream) with op COLL_ALLGATHER / COLL_ALLTOALL and device addresses.
    budget_gb > 0: the memory budget the plan must fit (every rank must pass
    the same: it sets the checkpoint count); 0: this device's free memory."""
    n, ev_v, ev_x = _ev(evidence)
    tg = list(range(model.n_vars)) if targets is None else list(targets)
    total = sum(model.cards[t] for t in tg)
    out = (C.c_double * max(total, 1))()
    exps = (C.c_int64 * max(len(tg), 1))()
    up = C.c_double()
    oa = _ints(list(order)) if order is not None else None
    h = ORDER_GIVEN if order is not None else HEURISTICS[heuristic]
    errors = []
    user = None
    if isinstance(collective, str) and collective.startswith("loopback"):
        # "loopback" (copies), "loopback-nocopy", "loopback-model:<MB/s per link>:<latency us>"
        # (no copies; each exchange's stream waits the modelled xGMI time)
        fn = COLLECTIVE_FN(C.cast(_lib.bnpp_collective_loopback, C.c_void_p).value)
        if collective.startswith("loopback-model"):
            _, rate, lat = collective.split(":")
            nr = (C.c_int * 4)(n_ranks, 3, int(rate), int(lat))
        else:
            nr = (C.c_int * 4)(n_ranks, 1 if collective == "loopback-nocopy" else 0, 0, 0)
        user = C.cast(nr, C.c_void_p)
    else:
        def _cb(_user, op, send, recv, nbytes, stream):
            try:
                collective(op, send, recv, nbytes, stream)
                return 0
            except BaseException as e:          # never unwind through the C frames
                errors.append(e)
                return 1
        fn = COLLECTIVE_FN(_cb)
    rc = _lib.bnpp_marginals_tree_sliced(ctx.handle, model.handle, n, ev_v, ev_x, h, oa,
                                         len(order) if order is not None else 0, len(tg), _ints(tg), rank, n_ranks,
                                         fn, user, C.c_double(budget_gb), dtype, out, exps, C.byref(up))
    if errors:
        raise errors[0]
    _check(rc, "bnpp_marginals_tree_sliced")
    mant, ex, o = {}, {}, 0
    for i, t in enumerate(tg):
        mant[t] = list(out[o:o + model.cards[t]])
        ex[t] = exps[i]
        o += model.cards[t]
    return mant, ex, up.value


def plan_tree_sliced(model: Model, rank: int, n_ranks: int, evidence=None, heuristic: str = "mf", dtype: int = F32,
                     order: Optional[Sequence[int]] = None):
    """Host-only plan of one rank of the sliced bucket tree -> (slice bit per
    variable, stats: Job's 8 then [8] exchanges, [9] bytes sent per call)."""
    n, ev_v, ev_x = _ev(evidence)
    sb = (C.c_int * max(model.n_vars, 1))()
    st = (C.c_double * 10)()
    oa = _ints(list(order)) if order is not None else None
    h = ORDER_GIVEN if order is not None else HEURISTICS[heuristic]
    _check(_lib.bnpp_plan_tree_sliced(model.handle, n, ev_v, ev_x, h, oa, len(order) if order is not None else 0,
                                      rank, n_ranks, dtype, sb, st, 10), "bnpp_plan_tree_sliced")
    return list(sb)[:model.n_vars], list(st)


def variable_elimination(ctx: Context, model: Model, variables: Sequence[int], heuristic: str = "given",
                         dtype: int = F64, cap_values: int = 1 << 20):
    """BN::variable_elimination over the model's factors as given ->
    (scope, values (scaled), exp2): true value = values * 2**exp2."""
    variables = list(variables)
    cap_vars = model.n_vars + 1
    ov = (C.c_int * cap_vars)()
    nd = C.c_int()
    size, e2 = C.c_int64(), C.c_int64()
    vals = (C.c_double * cap_values)()
    _check(_lib.bnpp_variable_elimination(ctx.handle, model.handle, len(variables), _ints(variables),
                                          HEURISTICS[heuristic], dtype, cap_vars, C.byref(nd), ov, cap_values,
                                          C.byref(size), vals, C.byref(e2)), "bnpp_variable_elimination")
    return list(ov[: nd.value]), list(vals[: size.value]), e2.value


class Job:
    """A prepared, device-resident inference (bnpp_job_*): launch() only enqueues."""

    def __init__(self, ctx: Context, model: Model, kind: str = "pr", evidence=None, heuristic: str = "mf",
                 dtype: int = F64, order: Optional[Sequence[int]] = None, targets: Optional[Sequence[int]] = None):
        n, ev_v, ev_x = _ev(evidence)
        self.model = model
        self.kind = {"pr": 0, "mar": 1, "mar_tree": 3}[kind]
        self.targets = list(range(model.n_vars)) if targets is None else list(targets)
        self._h = _P()
        order_arr = _ints(order) if order is not None else None
        h = ORDER_GIVEN if order is not None else HEURISTICS[heuristic]
        _check(_lib.bnpp_job_create(ctx.handle, model.handle, self.kind, n, ev_v, ev_x, h, order_arr,
                                    len(order) if order is not None else 0, len(self.targets), _ints(self.targets),
                                    dtype, C.byref(self._h)), "bnpp_job_create")
        st = (C.c_double * 8)()
        _check(_lib.bnpp_job_stats(self._h, st, 8), "bnpp_job_stats")
        (self.entries, self.arena_bytes, self.levels, self.buckets, self.width, self.max_table,
         self.alg_bytes, self.batches) = st[0], st[1], int(st[2]), int(st[3]), int(st[4]), st[5], st[6], int(st[7])

    def launch(self, stream: Optional[int] = None) -> None:
        _check(_lib.bnpp_job_launch(self._h, _P(stream) if stream else None), "bnpp_job_launch")

    def results(self, stream: Optional[int] = None):
        if self.kind == 0:
            out = (C.c_double * 1)()
            _check(_lib.bnpp_job_results(self._h, _P(stream) if stream else None, out), "bnpp_job_results")
            return out[0]
        total = sum(self.model.cards[t] for t in self.targets)
        out = (C.c_double * max(total, 1))()
        _check(_lib.bnpp_job_results(self._h, _P(stream) if stream else None, out), "bnpp_job_results")
        res, o = {}, 0
        for t in self.targets:
            res[t] = list(out[o:o + self.model.cards[t]])
            o += self.model.cards[t]
        return res

    def close(self):
        if self._h:
            _lib.bnpp_job_free(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bucket_eliminate(ctx: Context, dtype: int, cards: Sequence[int], tables: Sequence[int],
                     scopes: Sequence[Sequence[int]], elim: int, out: int, out_vars: Sequence[int],
                     stream: Optional[int] = None, out_sum: Optional[int] = None) -> None:
    """Fused bucket on caller-owned device buffers (addresses as ints, e.g. torch
    tensor.data_ptr()).  Only enqueues on `stream`.  out_sum: device address of
    a float64 that receives the reference's partition sum (include/bnpp.h)."""
    arrs = [_ints(s) for s in scopes]
    ptrs = (_IP * len(arrs))(*[C.cast(a, _IP) for a in arrs])
    tabs = (_P * len(tables))(*[_P(t) for t in tables])
    _check(_lib.bnpp_bucket_eliminate(ctx.handle, _P(stream) if stream else None, dtype, len(cards), _ints(cards), len(tables),
                                      tabs, _ints([len(s) for s in scopes]), ptrs, elim, _P(out), len(out_vars),
                                      _ints(out_vars), _P(out_sum) if out_sum else None), "bnpp_bucket_eliminate")


def divide(ctx: Context, dtype: int, cards: Sequence[int], a: int, a_scope: Sequence[int], b: int,
           b_scope: Sequence[int], out: int, out_vars: Sequence[int], stream: Optional[int] = None,
           out_sum: Optional[int] = None) -> None:
    """Factor::divide (factor.cpp:149-180) on caller-owned device buffers:
    out = a / b over the union scope (out_vars in any order of it)."""
    _check(_lib.bnpp_divide(ctx.handle, _P(stream) if stream else None, dtype, len(cards), _ints(cards), _P(a), len(a_scope),
                            _ints(a_scope), _P(b), len(b_scope), _ints(b_scope), _P(out), len(out_vars),
                            _ints(out_vars), _P(out_sum) if out_sum else None), "bnpp_divide")


def condition(ctx: Context, dtype: int, cards: Sequence[int], table: int, scope: Sequence[int],
              evidence: Dict[int, int], out: int, stream: Optional[int] = None, out_sum: Optional[int] = None) -> None:
    n, ev_v, ev_x = _ev(evidence)
    _check(_lib.bnpp_condition(ctx.handle, _P(stream) if stream else None, dtype, len(cards), _ints(cards), _P(table), len(scope),
                               _ints(scope), n, ev_v, ev_x, _P(out), _P(out_sum) if out_sum else None), "bnpp_condition")
