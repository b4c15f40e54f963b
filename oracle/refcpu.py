"""ctypes wrapper of the CPU restatement (oracle/refcpu.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker / CPU baseline, never by the
product path (bn-pp_amd/).  Build with `make -C oracle`.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "librefcpu.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")

GIVEN, MIN_FILL, WEIGHTED_MIN_FILL, MIN_DEGREE = 0, 1, 2, 3
HEURISTICS = {"given": GIVEN, "mf": MIN_FILL, "wmf": WEIGHTED_MIN_FILL, "md": MIN_DEGREE}

_lib = C.CDLL(LIB_PATH)
_P, _I, _IP, _DP = C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)
for name, res, args in [
    ("rc_factor_new", _P, [_I, _IP, _IP, _DP]),
    ("rc_factor_free", None, [_P]),
    ("rc_factor_width", _I, [_P]),
    ("rc_factor_size", C.c_uint64, [_P]),
    ("rc_factor_scope", None, [_P, _IP]),
    ("rc_factor_values", None, [_P, _DP]),
    ("rc_factor_partition", C.c_double, [_P]),
    ("rc_product", _P, [_P, _P]),
    ("rc_divide", _P, [_P, _P]),
    ("rc_sum_out", _P, [_P, _I, _I]),
    ("rc_conditioning", _P, [_P, _I, _IP, _IP]),
    ("rc_normalize", _P, [_P]),
    ("rc_bucket", _P, [_I, C.POINTER(_P), _I, _I]),
    ("rc_model_load_uai", _P, [C.c_char_p]),
    ("rc_model_new", _P, [_I, _I, _IP, _I, _IP, _IP, _DP]),
    ("rc_model_free", None, [_P]),
    ("rc_model_n_vars", _I, [_P]),
    ("rc_model_card", _I, [_P, _I]),
    ("rc_load_evidence", _I, [C.c_char_p, _I, _IP, _IP]),
    ("rc_partition", C.c_double, [_P, _I, _IP, _IP, _I, _DP]),
    ("rc_marginals", _I, [_P, _I, _IP, _IP, _I, _DP, _DP]),
    ("rc_marginal_one", _I, [_P, _I, _IP, _IP, _I, _I, _DP]),
    ("rc_micro_bucket", C.c_double, [_I, _I, _I, _DP]),
    ("rc_sum_product", _I, [_P, _I, C.c_double, _DP, _IP, _DP]),
    ("rc_ordering", _I, [_P, _I, C.POINTER(_P), _I, _IP, _I, _IP]),
    ("rc_variable_elimination", _P, [_P, _I, _IP, _I, C.POINTER(_P), _I]),
]:
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = args


def _ints(xs):
    xs = list(xs)
    return (C.c_int * max(len(xs), 1))(*xs)


def _dbls(xs):
    xs = list(xs)
    return (C.c_double * max(len(xs), 1))(*xs)


class Factor:
    """Owned rc_factor."""

    def __init__(self, h):
        self.h = h

    @classmethod
    def new(cls, scope: Sequence[int], cards_by_var: Dict[int, int], values: Sequence[float]) -> "Factor":
        return cls(_lib.rc_factor_new(len(scope), _ints(scope), _ints([cards_by_var[v] for v in scope]),
                                      _dbls(values)))

    @property
    def scope(self) -> List[int]:
        w = _lib.rc_factor_width(self.h)
        out = (C.c_int * max(w, 1))()
        _lib.rc_factor_scope(self.h, out)
        return list(out[:w])

    @property
    def values(self) -> List[float]:
        n = _lib.rc_factor_size(self.h)
        out = (C.c_double * max(n, 1))()
        _lib.rc_factor_values(self.h, out)
        return list(out[:n])

    @property
    def partition(self) -> float:
        return _lib.rc_factor_partition(self.h)

    def product(self, other: "Factor") -> "Factor":
        return Factor(_lib.rc_product(self.h, other.h))

    def divide(self, other: "Factor") -> "Factor":
        return Factor(_lib.rc_divide(self.h, other.h))

    def sum_out(self, var: int, card: int = 0) -> "Factor":
        return Factor(_lib.rc_sum_out(self.h, var, card))

    def conditioning(self, evidence: Dict[int, int]) -> "Factor":
        ks = sorted(evidence)
        return Factor(_lib.rc_conditioning(self.h, len(ks), _ints(ks), _ints([evidence[k] for k in ks])))

    def normalize(self) -> "Factor":
        return Factor(_lib.rc_normalize(self.h))

    def __del__(self):
        if self.h:
            _lib.rc_factor_free(self.h)
            self.h = None


def bucket(factors: Sequence[Factor], var: int, card: int = 0) -> Factor:
    arr = (_P * max(len(factors), 1))(*[f.h for f in factors])
    return Factor(_lib.rc_bucket(len(factors), arr, var, card))


class Model:
    def __init__(self, h):
        if not h:
            raise IOError("refcpu: cannot load model")
        self.h = h
        self.n_vars = _lib.rc_model_n_vars(h)
        self.cards = [_lib.rc_model_card(h, v) for v in range(self.n_vars)]

    @classmethod
    def load(cls, path: str) -> "Model":
        return cls(_lib.rc_model_load_uai(path.encode()))

    @classmethod
    def from_dict(cls, m: dict) -> "Model":
        widths = [len(s) for s in m["scopes"]]
        return cls(_lib.rc_model_new(1 if m.get("type") == "BAYES" else 0, len(m["cards"]), _ints(m["cards"]),
                                     len(widths), _ints(widths), _ints([v for s in m["scopes"] for v in s]),
                                     _dbls([x for vals in m["values"] for x in vals])))

    def __del__(self):
        if self.h:
            _lib.rc_model_free(self.h)
            self.h = None

    def _ev(self, evidence):
        evidence = evidence or {}
        ks = sorted(evidence)
        return len(ks), _ints(ks), _ints([evidence[k] for k in ks])

    def partition(self, evidence=None, heuristic: str = "mf"):
        """-> (Z, uptime_ms)"""
        n, v, x = self._ev(evidence)
        up = C.c_double()
        z = _lib.rc_partition(self.h, n, v, x, HEURISTICS[heuristic], C.byref(up))
        return z, up.value

    def marginals(self, evidence=None, heuristic: str = "mf"):
        n, v, x = self._ev(evidence)
        total = sum(self.cards)
        out = (C.c_double * max(total, 1))()
        up = C.c_double()
        _lib.rc_marginals(self.h, n, v, x, HEURISTICS[heuristic], out, C.byref(up))
        res, o = {}, 0
        for t in range(self.n_vars):
            res[t] = list(out[o:o + self.cards[t]])
            o += self.cards[t]
        return res, up.value

    def sum_product(self, max_iter: int = 10000, eps: float = 0.001):
        """Loopy BP (model.cpp:313-317, 736-753) -> (marginals {var: [..]}, iterations, uptime_ms)."""
        out = (C.c_double * max(sum(self.cards), 1))()
        it, up = C.c_int(), C.c_double()
        _lib.rc_sum_product(self.h, max_iter, eps, out, C.byref(it), C.byref(up))
        res, o = {}, 0
        for t in range(self.n_vars):
            res[t] = list(out[o:o + self.cards[t]])
            o += self.cards[t]
        return res, it.value, up.value

    def ordering(self, variables: Sequence[int], heuristic: str = "mf"):
        """Graph::ordering over the model's own (unconditioned) factors -> (order, width)."""
        nf = _lib_model_nf(self.h)
        fs = C.cast(C.c_void_p(_model_factors(self.h)), C.POINTER(_P))
        out = (C.c_int * max(len(variables), 1))()
        w = _lib.rc_ordering(self.h, nf, fs, len(variables), _ints(variables), HEURISTICS[heuristic], out)
        return list(out[:len(variables)]), w

    def variable_elimination(self, variables: Sequence[int], heuristic: str = "given") -> "Factor":
        """BN::variable_elimination (model.cpp:348-446) over the model's own
        factors, eliminating `variables` (in this order with "given")."""
        nf = _lib_model_nf(self.h)
        fs = C.cast(C.c_void_p(_model_factors(self.h)), C.POINTER(_P))
        variables = list(variables)
        return Factor(_lib.rc_variable_elimination(self.h, len(variables), _ints(variables), nf, fs,
                                                   HEURISTICS[heuristic]))

    def marginal(self, target: int, evidence=None, heuristic: str = "mf"):
        n, v, x = self._ev(evidence)
        out = (C.c_double * self.cards[target])()
        _lib.rc_marginal_one(self.h, n, v, x, HEURISTICS[heuristic], target, out)
        return list(out)


class _RcModel(C.Structure):
    _fields_ = [("is_bayes", C.c_int), ("n_vars", C.c_int), ("cards", _IP), ("n_factors", C.c_int),
                ("factors", C.c_void_p)]


def _lib_model_nf(h) -> int:
    return C.cast(C.c_void_p(h), C.POINTER(_RcModel)).contents.n_factors


def _model_factors(h) -> int:
    return C.cast(C.c_void_p(h), C.POINTER(_RcModel)).contents.factors


def load_evidence(path: str) -> Dict[int, int]:
    cap = 1 << 16
    vs, xs = (C.c_int * cap)(), (C.c_int * cap)()
    n = _lib.rc_load_evidence(path.encode(), cap, vs, xs)
    if n < 0:
        raise IOError(path)
    return {vs[i]: xs[i] for i in range(n)}


def micro_bucket(k: int, w: int, reps: int = 1):
    """-> (factor-entries/s, seconds) of the restated m(x,S)*f(x,y) -> sum_x bucket."""
    sec = C.c_double()
    eps = _lib.rc_micro_bucket(k, w, reps, C.byref(sec))
    return eps, sec.value
