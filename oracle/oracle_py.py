"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY -- see oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        P, I, D, L64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int64
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        sig = {
            "oracle_create": (P, [I, I, I, D, I, I, I]),
            "oracle_destroy": (None, [P]),
            "oracle_num_nodes": (L64, [P]),
            "oracle_get_nodes": (None, [P, dp]),
            "oracle_get_weights": (None, [P, dp]),
            "oracle_set_coeff": (None, [P, dp, dp]),
            "oracle_cache": (None, [P, I]),
            "oracle_uncache": (None, [P, I]),
            "oracle_mapping": (None, [P, dp, I, dp]),
            "oracle_mapping_stages": (None, [P, dp, I, dp]),
            "oracle_set_faithful_rebuild": (None, [P, I]),
            "oracle_set_reference_alloc": (None, [P, I]),
            "oracle_gmres_main": (I, [P, dp, dp, I, I, D, dp, I, dp]),
            "oracle_refine_size": (I, [P]),
            "oracle_get_matrices": (None, [P, dp, dp, dp, dp]),
            "oracle_line_integral": (D, [P, D, D, D, D]),
            "oracle_eval_kernel": (D, [P, I, I, D, D, D, D]),
            "otree_build": (P, [dp, dp, I, I, I]),
            "otree_destroy": (None, [P]),
            "otree_num_nodes": (I, [P]),
            "otree_max_level": (I, [P]),
            "otree_node_ints": (None, [P, I, ip]),
            "otree_node_geom": (None, [P, I, dp]),
            "otree_list": (I, [P, I, I, ip]),
            "otree_sources": (I, [P, I, ip]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


class Oracle:
    """Mirror of the reference MATLAB class Aniso (class/@Aniso/Aniso.m:1-34)."""

    def __init__(self, sz, d, ks, g, ns, np_, maxLevel):
        self.h = lib().oracle_create(sz, d, ks, g, ns, np_, maxLevel)
        self.N = int(lib().oracle_num_nodes(self.h))
        self.sz, self.d, self.ks, self.ns = sz, d, ks, ns

    def close(self):
        if self.h:
            lib().oracle_destroy(self.h)
            self.h = None

    __del__ = close

    def getNodes(self):
        xy = np.zeros(2 * self.N)
        lib().oracle_get_nodes(self.h, _dp(xy))
        return xy.reshape(2, self.N).T.copy()

    def weights(self):
        w = np.zeros(self.N)
        lib().oracle_get_weights(self.h, _dp(w))
        return w

    def setCoeff(self, sigma_s, sigma_t):
        s = np.ascontiguousarray(sigma_s, dtype=np.float64)
        t = np.ascontiguousarray(sigma_t, dtype=np.float64)
        lib().oracle_set_coeff(self.h, _dp(s), _dp(t))

    def cache(self, mode):
        lib().oracle_cache(self.h, int(mode))

    def uncache(self, mode):
        lib().oracle_uncache(self.h, int(mode))

    def mapping(self, charge, mode):
        c = np.ascontiguousarray(charge, dtype=np.float64)
        out = np.zeros(self.N)
        lib().oracle_mapping(self.h, _dp(c), int(mode), _dp(out))
        return out

    def mapping_stages(self, charge, mode):
        c = np.ascontiguousarray(charge, dtype=np.float64)
        st = np.zeros(6 * self.N)
        lib().oracle_mapping_stages(self.h, _dp(c), int(mode), _dp(st))
        return st.reshape(6, self.N)

    def set_faithful(self, on):
        lib().oracle_set_faithful_rebuild(self.h, int(on))

    def set_reference_alloc(self, on):
        """Timing mode: the reference's per-use heap Vectors / block copies (same results)."""
        lib().oracle_set_reference_alloc(self.h, int(on))

    def gmres_main(self, q, m=80, maxit=400, tol=1e-12, x0=None):
        q = np.ascontiguousarray(q, dtype=np.float64)
        x = np.zeros(self.N) if x0 is None else np.array(x0, dtype=np.float64)
        hist = np.zeros(maxit + 2)
        fr = np.zeros(1)
        j = lib().oracle_gmres_main(self.h, _dp(q), _dp(x), m, maxit, tol, _dp(hist), len(hist), _dp(fr))
        return j, x, hist, float(fr[0])

    def line_integral(self, x0, y0, x1, y1):
        return lib().oracle_line_integral(self.h, x0, y0, x1, y1)

    def eval_kernel(self, imag, mode, a, b):
        return lib().oracle_eval_kernel(self.h, int(imag), int(mode), a[0], a[1], b[0], b[1])

    def matrices(self):
        d2 = self.d * self.d
        nref = lib().oracle_refine_size(self.h)
        interp = np.zeros(d2 * d2)
        nm = np.zeros(nref * d2)
        ln = np.zeros(d2)
        sw = np.zeros(d2)
        lib().oracle_get_matrices(self.h, _dp(interp), _dp(nm), _dp(ln), _dp(sw))
        return (interp.reshape(d2, d2, order="F"), nm.reshape(nref, d2, order="F"), ln, sw)


class OTree:
    """Standalone restatement of bbfmm::tree::populate (bbfmm.h:176-413)."""

    def __init__(self, x, y, rank=16, maxLevel=20):
        self.x = np.ascontiguousarray(x, dtype=np.float64)
        self.y = np.ascontiguousarray(y, dtype=np.float64)
        self.h = lib().otree_build(_dp(self.x), _dp(self.y), len(self.x), rank, maxLevel)
        self.nn = lib().otree_num_nodes(self.h)

    def close(self):
        if self.h:
            lib().otree_destroy(self.h)
            self.h = None

    __del__ = close

    @property
    def max_level(self):
        return lib().otree_max_level(self.h)

    def node_ints(self):
        out = np.zeros((self.nn, 11), dtype=np.int32)
        buf = np.zeros(11, dtype=np.int32)
        for i in range(self.nn):
            lib().otree_node_ints(self.h, i, _ip(buf))
            out[i] = buf
        return out  # parent, child0..3, level, slot, isLeaf, isEmpty, nSource, 0

    def node_geom(self):
        out = np.zeros((self.nn, 4))
        buf = np.zeros(4)
        for i in range(self.nn):
            lib().otree_node_geom(self.h, i, _dp(buf))
            out[i] = buf
        return out

    def lists(self, which):
        """which: 0=U 1=V 2=W 3=X -> list of sorted int arrays."""
        res = []
        for i in range(self.nn):
            n = lib().otree_list(self.h, i, which, None)
            a = np.zeros(n, dtype=np.int32)
            if n:
                lib().otree_list(self.h, i, which, _ip(a))
            res.append(a)
        return res

    def sources(self, i):
        n = lib().otree_sources(self.h, i, None)
        a = np.zeros(n, dtype=np.int32)
        if n:
            lib().otree_sources(self.h, i, _ip(a))
        return a
