"""aniso_amd -- MI355X-native matvec of the lowrank/aniso anisotropic RTE solver.

Host-side mirror of the reference's plugin interface: the MATLAB handle class
`Aniso` (class/@Aniso/Aniso.m:1-34) over the MEX ops new/delete/getNodes/
setCoeff/cache/mapping (AnisoWrapper.cpp:10-136).  Everything here calls the C ABI
of `libaniso_mi355x.so` (include/aniso_mi355x.h); the compute runs in the HIP
kernels of aniso_amd/csrc.  There is no CPU fallback: a missing library or a
missing GPU raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ANISO_LIB") or os.path.join(_HERE, "libaniso_mi355x.so")  # ANISO_LIB: dev builds
_lib = None

STAGE_FAR, STAGE_NEAR, STAGE_STENCIL, STAGE_SING, STAGE_ALL = 1, 2, 4, 8, 15


# the caller-supplied collectives of the library's multi-GPU exchange (aniso_collectives)
COLL_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_void_p)
COLL_ALLTOALLV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                  ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                  ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p)
COLL_ALLREDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


class Collectives(ctypes.Structure):
    """aniso_collectives (include/aniso_mi355x.h)."""

    _fields_ = [("ctx", ctypes.c_void_p), ("allgather", COLL_ALLGATHER), ("alltoallv", COLL_ALLTOALLV),
                ("allreduce", COLL_ALLREDUCE)]


class AnisoError(RuntimeError):
    """Raised for any non-zero status of the C ABI (mexErrMsgIdAndTxt analogue)."""

    def __init__(self, code, msg):
        super().__init__(f"[aniso status {code}] {msg}")
        self.code = code


def lib():
    """Load the C ABI library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # PyTorch-ROCm ships its own libamdhip64.so.7; load it first so that this
        # library binds to the same HIP runtime (same SONAME) instead of a second
        # copy from /opt/rocm -- two runtimes in one process cannot share a GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise AnisoError(-1, f"{LIB_PATH} not built; run `make -C aniso_amd/csrc`")
        L = ctypes.CDLL(LIB_PATH)
        P, I, D, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int64
        dp, ip, lp = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64)
        fp = ctypes.POINTER(ctypes.c_float)
        sig = {
            "aniso_create": [I, I, I, D, I, I, I, ctypes.POINTER(P)],
            "aniso_destroy": [P],
            "aniso_num_nodes": [P, lp],
            "aniso_num_blocks": [P, ip],
            "aniso_sync": [P],
            "aniso_get_nodes": [P, dp],
            "aniso_get_weights": [P, dp],
            "aniso_set_coeff": [P, dp, dp],
            "aniso_cache": [P, I],
            "aniso_mapping": [P, dp, I, dp],
            "aniso_mapping_dev": [P, P, I, P, P],
            "aniso_mapping_batched": [P, dp, I, I, dp],
            "aniso_mapping_stages_dev": [P, P, I, I, P, P],
            "aniso_set_shard": [P, I, I],
            "aniso_get_shard": [P, lp, lp],
            "aniso_tree_perm": [P, ip],
            "aniso_permute_to_tree_dev": [P, P, P, P],
            "aniso_tree_size": [P, ip, ip],
            "aniso_tree_nodes": [P, ip, dp],
            "aniso_tree_list": [P, I, lp, ip],
            "aniso_stats": [P, lp],
            "aniso_stats_n": [P, lp, I, ip],
            "aniso_set_timing": [P, I],
            "aniso_stage_times": [P, fp],
            "aniso_line_integrals": [P, dp, I, dp],
            "aniso_top_trace": [P, lp, I64, lp],
            "aniso_forward_dev": [P, P, P, P],
            "aniso_mapping_tree_dev": [P, P, I, P, P],
            "aniso_forward_tree_dev": [P, P, P, P],
            "aniso_gmres": [P, dp, dp, I, I, D, dp, I, ip, dp],
            "aniso_block_solve": [P, dp, dp, I, D, I, dp, I, ip, dp],
            "aniso_block_solve_dev": [P, P, P, I, D, I, dp, I, ip, dp, P],
            "aniso_solve16_mixed_dev": [P, P, I64, P, I64, I, D, D, I, I, ip, ip, dp, P],
            "aniso_apply_block_dev": [P, I, P, I64, I, I, ip, dp, P, I64, I, P],
            "aniso_block_op_dev": [P, I, P, I64, P, I64, I, P],
            "aniso_block_mixes": [I, D, I, dp],
            "aniso_block_op": [P, I, dp, dp],
            "aniso_apply_block": [P, dp, dp, D, dp],
            "aniso_shard_cuts": [P, I, lp],
            "aniso_forward_f32_dev": [P, P, P, P],
            "aniso_forward16_f64_dev": [P, P, P, P],
            "aniso_mapping16_f64_dev": [P, I, P, P, I, P],
            "aniso_forward_f32_stages_dev": [P, P, I, P, P],
            "aniso_set_deterministic": [P, I],
            "aniso_shard_exchange": [P, I, lp],
            "aniso_shard_exchange_one": [P, lp],
            "aniso_shard_one_halo": [P, lp],
            "aniso_shard_upper_partials": [P, lp],
            "aniso_shard_upper_records": [P, ip],
            "aniso_shard_halo": [P, lp],
            "aniso_shard_roots": [P, ip, ip, ip],
            "aniso_forward_tree_begin_dev": [P, P, P, P, P],
            "aniso_forward_tree_end_dev": [P, P, P, P, P],
            "aniso_block_op_begin_dev": [P, I, P, I64, P, I64, P, P],
            "aniso_block_op_end_dev": [P, I, P, I64, P, I64, P, P],
            "aniso_last_error": [ctypes.c_char_p, ctypes.c_size_t],
            "aniso_comm_unique_id": [ctypes.c_char_p],
            "aniso_comm_init_rccl": [P, ctypes.c_char_p],
            "aniso_comm_init_callbacks": [P, ctypes.POINTER(Collectives)],
            "aniso_comm_init_loopback": [P],
            "aniso_krylov_dot": [P, I64, I, P, I64, P, P, P],
            "aniso_krylov_update": [P, I64, I, P, I64, P, P, P, I, P],
            "aniso_block_op_sharded_dev": [P, I, P, I64, P, I64, P],
            "aniso_arnoldi_state_size": [I, lp],
            "aniso_arnoldi_begin": [P, I64, I, P, I64, P, P, D, P, P],
            "aniso_arnoldi_step": [P, I64, I, I, P, I64, P, P, P, P],
            "aniso_arnoldi_project": [P, I64, I, P, I64, P, P, P],
            "aniso_arnoldi_coef": [P, I, I, P, P, P],
            "aniso_arnoldi_update": [P, I64, I, I, P, I64, P, P, P, P],
            "aniso_arnoldi_column": [P, I, I, P, P, P, P],
            "aniso_arnoldi_solution": [P, I64, I, I, P, I64, P, P, P],
            "aniso_mapped_alloc": [ctypes.c_size_t, ctypes.POINTER(P), ctypes.POINTER(P)],
            "aniso_mapped_free": [P],
            "aniso_memcpy": [P, P, ctypes.c_size_t],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = I
        L.aniso_version.restype = ctypes.c_char_p
        L.aniso_version.argtypes = []
        _lib = L
    return _lib


def exported_symbols(public_only=False):
    """Names of the entry points declared in include/aniso_mi355x.h (the drop-in
    boundary) and, unless public_only, include/aniso_mi355x_dev.h (development and
    test entries)."""
    heads = ["aniso_mi355x.h"] + ([] if public_only else ["aniso_mi355x_dev.h"])
    hdr = "".join(open(os.path.join(_HERE, "..", "include", h)).read() for h in heads)
    import re

    return sorted(set(re.findall(r"^(?:int|const char \*)\s*\**\s*(aniso_\w+)\s*\(", hdr, re.M)))


def _check(code):
    if code != 0:
        buf = ctypes.create_string_buffer(4096)
        lib().aniso_last_error(buf, len(buf))
        raise AnisoError(code, buf.value.decode(errors="replace"))


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _f64(a, n, name):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
    if a.size != n:
        raise AnisoError(1, f"{name} has {a.size} entries, expected N = {n}")
    return a


def _dev_vec(t, n, name, at_least=False):
    """A contiguous float64 CUDA tensor of n entries (at least n for an output slice
    the kernels fill from the front; else AnisoError)."""
    import torch

    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
            and (t.numel() >= n if at_least else t.numel() == n)):
        raise AnisoError(1, f"{name} must be a contiguous float64 CUDA tensor of {'>= ' if at_least else ''}{n} entries")
    return ctypes.c_void_p(t.data_ptr())


def _krylov_args(V, w, out, nout):
    import torch

    for name, t in (("V", V), ("w", w), ("out", out)):
        if not (t.is_cuda and t.dtype == torch.float64):
            raise ValueError(f"{name}: float64 CUDA tensor expected")
    if V.dim() != 2 or V.stride(1) != 1 or V.shape[0] < 1:
        raise ValueError("V: (nv, n) with unit inner stride")
    if not (w.is_contiguous() and w.numel() == V.shape[1]):
        raise ValueError("w: contiguous, n entries")
    if not (out.is_contiguous() and out.numel() >= nout):
        raise ValueError(f"out: contiguous, >= {nout} entries")


def _dev_rows(t, rows, cols, name):
    """A float64 CUDA tensor of `rows` rows of at least `cols` entries (unit column
    stride, row stride >= cols): the kernels touch the first cols of every row."""
    import torch

    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.dim() == 2
            and t.stride(1) == 1 and t.shape[0] == rows and t.shape[1] >= cols and (rows == 1 or t.stride(0) >= cols)):
        raise AnisoError(1, f"{name} must be a ({rows}, >= {cols}) float64 CUDA tensor with unit column stride")
    return ctypes.c_void_p(t.data_ptr())


class MappedStatus:
    """A few doubles of pinned host memory mapped into the device (aniso_mapped_alloc):
    kernels store a status word through .dev, the host reads .host after an event."""

    def __init__(self, n=4):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _check(lib().aniso_mapped_alloc(8 * n, ctypes.byref(h), ctypes.byref(d)))
        self._h, self.dev, self.n = h, d, n
        self.host = np.ctypeslib.as_array(ctypes.cast(h, ctypes.POINTER(ctypes.c_double)), shape=(n,))

    def close(self):
        if self._h:
            lib().aniso_mapped_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Aniso:
    """Aniso(ds, qr, ks, as, sr, fn, fm) -- class/@Aniso/Aniso.m:8-11.

    ds: squares per side, qr: quadrature rule, ks: kernel size (modes 0..2ks-2),
    as: anisotropy g, sr: singular rule, fn: FMM np (4), fm: FMM maxLevel.
    """

    def __init__(self, ds, qr, ks, as_, sr, fn, fm):
        h = ctypes.c_void_p()
        _check(lib().aniso_create(int(ds), int(qr), int(ks), float(as_), int(sr), int(fn), int(fm), ctypes.byref(h)))
        self.address = h
        n = ctypes.c_int64()
        _check(lib().aniso_num_nodes(h, ctypes.byref(n)))
        self.N = n.value
        self.sz, self.d, self.ks, self.g, self.ns, self.np, self.maxLevel = int(ds), int(qr), int(ks), float(as_), int(sr), int(fn), int(fm)

    # 'delete' (Aniso.m:13-16)
    def close(self):
        if getattr(self, "address", None):
            lib().aniso_destroy(self.address)
            self.address = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def getNodes(self):
        """N x 2 array of quadrature nodes (Aniso.m:22-24)."""
        xy = np.zeros(2 * self.N)
        _check(lib().aniso_get_nodes(self.address, _dp(xy)))
        return xy.reshape(2, self.N).T.copy()

    def getWeights(self):
        w = np.zeros(self.N)
        _check(lib().aniso_get_weights(self.address, _dp(w)))
        return w

    def setCoeff(self, sigma_s, sigma_t):
        """Aniso.m:18-20."""
        s = _f64(sigma_s, self.N, "sigma_s")
        t = _f64(sigma_t, self.N, "sigma_t")
        _check(lib().aniso_set_coeff(self.address, _dp(s), _dp(t)))

    def cache(self, id_):
        """Aniso.m:26-28."""
        _check(lib().aniso_cache(self.address, int(id_)))

    def mapping(self, charge, id_):
        """Aniso.m:30-32: returns K_id * charge (N,)."""
        c = _f64(charge, self.N, "charge")
        out = np.zeros(self.N)
        _check(lib().aniso_mapping(self.address, _dp(c), int(id_), _dp(out)))
        return out

    def mapping_batched(self, Q, id_):
        Q = np.asfortranarray(np.asarray(Q, dtype=np.float64))
        if Q.ndim != 2 or Q.shape[0] != self.N:
            raise AnisoError(1, f"Q must be N x k with N = {self.N}")
        out = np.zeros(Q.shape, order="F")
        _check(lib().aniso_mapping_batched(self.address, _dp(Q), Q.shape[1], int(id_), _dp(out)))
        return out

    # ---- device-pointer variants (torch tensors on the current HIP device)
    def mapping_dev(self, charge, id_, out, stream=None, mask=STAGE_ALL):
        """charge/out: contiguous float64 torch tensors of N entries on the GPU."""
        import torch

        _dev_vec(charge, self.N, "charge")
        _dev_vec(out, self.N, "out")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        if mask == STAGE_ALL:
            _check(lib().aniso_mapping_dev(self.address, ctypes.c_void_p(charge.data_ptr()), int(id_),
                                           ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s)))
        else:
            _check(lib().aniso_mapping_stages_dev(self.address, ctypes.c_void_p(charge.data_ptr()), int(id_), int(mask),
                                                  ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s)))
        return out

    def forward_dev(self, u, out, stream=None):
        """main.cpp forwardOperator on device tensors: out = u - K_0(sigma_s .* u)."""
        import torch

        pu, po = _dev_vec(u, self.N, "u"), _dev_vec(out, self.N, "out")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_forward_dev(self.address, pu, po, ctypes.c_void_p(s)))
        return out

    def mapping_tree_dev(self, q_tree, id_, out_slice, stream=None):
        """mapping on a tree-order device vector (all N) into the owned tree-order slice."""
        import torch

        pq, po = _dev_vec(q_tree, self.N, "q_tree"), _dev_vec(out_slice, self.n_owned(), "out_slice", True)
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_mapping_tree_dev(self.address, pq, int(id_), po, ctypes.c_void_p(s)))
        return out_slice

    def forward_tree_dev(self, x_tree, y_slice, stream=None):
        """forwardOperator in tree order: y_slice = (x - K_0(sigma_s .* x))[own slice], x tree-ordered."""
        import torch

        px, py = _dev_vec(x_tree, self.N, "x_tree"), _dev_vec(y_slice, self.n_owned(), "y_slice", True)
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_forward_tree_dev(self.address, px, py, ctypes.c_void_p(s)))
        return y_slice

    def forward_f32_dev(self, X, Y, stream=None, mask=STAGE_ALL):
        """Config 5's fp32 operator: Y = X - K_0(sigma_s .* X) for 16 right-hand sides on
        MFMA.  X, Y: (N, 16) contiguous float32 CUDA tensors, point-major, tree order."""
        import torch

        for t, nm in ((X, "X"), (Y, "Y")):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                    and tuple(t.shape) == (self.N, 16)):
                raise AnisoError(1, f"{nm} must be a contiguous ({self.N}, 16) float32 CUDA tensor")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        if mask == STAGE_ALL:
            _check(lib().aniso_forward_f32_dev(self.address, ctypes.c_void_p(X.data_ptr()),
                                               ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(s)))
        else:
            _check(lib().aniso_forward_f32_stages_dev(self.address, ctypes.c_void_p(X.data_ptr()), int(mask),
                                                      ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(s)))
        return Y

    def forward16_f64_dev(self, X, Y, stream=None):
        """The fp64 16-RHS operator on MFMA: Y = X - K_0(sigma_s .* X); X, Y (N, 16)
        contiguous float64 CUDA tensors, point-major, tree order."""
        import torch

        for t, nm in ((X, "X"), (Y, "Y")):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
                    and tuple(t.shape) == (self.N, 16)):
                raise AnisoError(1, f"{nm} must be a contiguous ({self.N}, 16) float64 CUDA tensor")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_forward16_f64_dev(self.address, ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(Y.data_ptr()),
                                             ctypes.c_void_p(s)))
        return Y

    def mapping16_f64_dev(self, id_, X, Y, mask=STAGE_ALL, stream=None):
        """Y = K_id X for 16 right-hand sides on fp64 MFMA (shapes as forward16_f64_dev)."""
        import torch

        for t, nm in ((X, "X"), (Y, "Y")):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
                    and tuple(t.shape) == (self.N, 16)):
                raise AnisoError(1, f"{nm} must be a contiguous ({self.N}, 16) float64 CUDA tensor")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_mapping16_f64_dev(self.address, int(id_), ctypes.c_void_p(X.data_ptr()),
                                             ctypes.c_void_p(Y.data_ptr()), int(mask), ctypes.c_void_p(s)))
        return Y

    # ---- the block operator of aniso.m (aniso.m:121-157)
    def apply_block_dev(self, x, ids, mixes, out, use_sigma=False, tree=False, stream=None):
        """out[i] = sum_t sum_b mixes[t][i][b] mapping(sig .* x[b], ids[t]) on device tensors.

        x: (nrhs, N) float64 CUDA tensor (rows may be strided); out: (nrhs, n_out)
        with n_out = N (original order) or the owned slice length (tree=True);
        mixes: (nterm, nrhs, nrhs) host array; use_sigma multiplies x by sigma_s.
        """
        import torch

        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int32).reshape(-1))
        nrhs = x.shape[0]
        mixes = np.ascontiguousarray(np.asarray(mixes, dtype=np.float64).reshape(len(ids), nrhs, nrhs))
        _dev_rows(x, nrhs, self.N, "x")
        _dev_rows(out, nrhs, self.n_owned() if tree else self.N, "out")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_apply_block_dev(self.address, int(nrhs), ctypes.c_void_p(x.data_ptr()), int(x.stride(0)),
                                           int(bool(use_sigma)), len(ids),
                                           ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _dp(mixes),
                                           ctypes.c_void_p(out.data_ptr()), int(out.stride(0)), int(bool(tree)),
                                           ctypes.c_void_p(s)))
        return out

    def block_op_dev(self, which, x, out, tree=False, stream=None):
        """aniso.m on ks stacked blocks: which = 0 forward, 1 mforward, 2 x - mforward(x).

        x: (ks, N) device tensor (block b = u(b*n+1:(b+1)*n)); out: (ks, n_out)."""
        import torch

        _dev_rows(x, self.ks, self.N, "x")
        _dev_rows(out, self.ks, self.n_owned() if tree else self.N, "out")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_block_op_dev(self.address, int(which), ctypes.c_void_p(x.data_ptr()), int(x.stride(0)),
                                        ctypes.c_void_p(out.data_ptr()), int(out.stride(0)), int(bool(tree)),
                                        ctypes.c_void_p(s)))
        return out

    # ---- sharded applies in two phases around the caller's root all-gather
    # (aniso_shard_exchange)
    def _roots_buf(self, t, n, name):
        if n == 0:
            return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None
        return _dev_vec(t, n, name, True)

    def block_op_begin_dev(self, which, x, out, roots_send, stream=None):
        """Phase 1 of the sharded x - mforward(x) etc.: x (ks, N) tree order, valid at
        the own range and the halo; out (ks, >= n_owned); roots_send >= C x R doubles."""
        import torch

        ex = self.shard_exchange(self.ks)
        _dev_rows(x, self.ks, self.N, "x")
        _dev_rows(out, self.ks, self.n_owned(), "out")
        rs = self._roots_buf(roots_send, ex["root_chunk"] * ex["root_record"], "roots_send")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_block_op_begin_dev(self.address, int(which), ctypes.c_void_p(x.data_ptr()),
                                              int(x.stride(0)), ctypes.c_void_p(out.data_ptr()), int(out.stride(0)),
                                              rs, ctypes.c_void_p(s)))

    def block_op_end_dev(self, which, x, out, roots_recv, nranks, stream=None):
        """Phase 2: roots_recv = the all-gather of every rank's roots_send (nranks x C x R)."""
        import torch

        ex = self.shard_exchange(self.ks)
        _dev_rows(x, self.ks, self.N, "x")
        _dev_rows(out, self.ks, self.n_owned(), "out")
        rr = self._roots_buf(roots_recv, nranks * ex["root_chunk"] * ex["root_record"], "roots_recv")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_block_op_end_dev(self.address, int(which), ctypes.c_void_p(x.data_ptr()), int(x.stride(0)),
                                            ctypes.c_void_p(out.data_ptr()), int(out.stride(0)), rr,
                                            ctypes.c_void_p(s)))
        return out

    def forward_tree_begin_dev(self, x_tree, y_slice, roots_send, stream=None):
        import torch

        ex = self.shard_exchange(1)
        px, py = _dev_vec(x_tree, self.N, "x_tree"), _dev_vec(y_slice, self.n_owned(), "y_slice", True)
        rs = self._roots_buf(roots_send, ex["root_chunk"] * ex["root_record"], "roots_send")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_forward_tree_begin_dev(self.address, px, py, rs, ctypes.c_void_p(s)))

    def forward_tree_end_dev(self, x_tree, y_slice, roots_recv, nranks, stream=None):
        import torch

        ex = self.shard_exchange(1)
        px, py = _dev_vec(x_tree, self.N, "x_tree"), _dev_vec(y_slice, self.n_owned(), "y_slice", True)
        rr = self._roots_buf(roots_recv, nranks * ex["root_chunk"] * ex["root_record"], "roots_recv")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_forward_tree_end_dev(self.address, px, py, rr, ctypes.c_void_p(s)))
        return y_slice

    def block_op(self, which, u):
        """aniso.m forward (0) / mforward (1) / x - mforward(x) (2) on host arrays:
        u is (ks, N) or the stacked ks*N column of aniso.m; returns (ks, N)."""
        u = _f64(u, self.ks * self.N, "u")
        out = np.zeros(self.ks * self.N)
        _check(lib().aniso_block_op(self.address, int(which), _dp(u), _dp(out)))
        return out.reshape(self.ks, self.N)

    def apply_block(self, u, sigma_s, g):
        """A(u) = u - mforward(u) with explicit sigma_s and g."""
        u = _f64(u, self.ks * self.N, "u")
        s = _f64(sigma_s, self.N, "sigma_s")
        out = np.zeros(self.ks * self.N)
        _check(lib().aniso_apply_block(self.address, _dp(u), _dp(s), float(g), _dp(out)))
        return out.reshape(self.ks, self.N)

    def gmres(self, q, m=80, maxit=400, tol=1e-12, x0=None):
        """main.cpp:121-141 on the device: returns (iters, x, residual history, final residual)."""
        q = _f64(q, self.N, "q")
        x = np.zeros(self.N) if x0 is None else _f64(x0, self.N, "x0").copy()
        hist = np.zeros(maxit + 2)
        it = ctypes.c_int()
        fr = ctypes.c_double()
        _check(lib().aniso_gmres(self.address, _dp(q), _dp(x), int(m), int(maxit), float(tol), _dp(hist), len(hist),
                                 ctypes.byref(it), ctypes.byref(fr)))
        n = abs(it.value) + 1 if it.value != 0 else 1
        return it.value, x, hist[:n], fr.value

    def block_solve(self, rhs, restart=400, tol=1e-11, maxit=400, x0=None):
        """aniso.m:159-173 on the device: u = gmres(A, rhs, restart, tol, maxit), A = u - mforward(u).
        rhs: (ks, N) or the stacked ks*N column; returns (iters, u (ks, N), residual history, relres)."""
        rhs = _f64(rhs, self.ks * self.N, "rhs")
        x = np.zeros(self.ks * self.N) if x0 is None else _f64(x0, self.ks * self.N, "x0").copy()
        hist = np.zeros(restart * maxit if restart * maxit < 100000 else 100000)
        it, rr = ctypes.c_int(), ctypes.c_double()
        _check(lib().aniso_block_solve(self.address, _dp(rhs), _dp(x), int(restart), float(tol), int(maxit), _dp(hist),
                                       len(hist), ctypes.byref(it), ctypes.byref(rr)))
        return it.value, x.reshape(self.ks, self.N), hist[: min(abs(it.value), len(hist))], rr.value

    def block_solve_dev(self, rhs, x, restart=400, tol=1e-11, maxit=400, stream=None):
        """The same on (ks, N) float64 CUDA tensors (original order); x: guess in, solution out."""
        import torch

        pr, px = _dev_vec(rhs, self.ks * self.N, "rhs"), _dev_vec(x, self.ks * self.N, "x")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        hist = np.zeros(min(restart * maxit, 100000))
        it, rr = ctypes.c_int(), ctypes.c_double()
        _check(lib().aniso_block_solve_dev(self.address, pr, px, int(restart), float(tol), int(maxit), _dp(hist),
                                           len(hist), ctypes.byref(it), ctypes.byref(rr), ctypes.c_void_p(s)))
        return it.value, hist[: min(abs(it.value), len(hist))], rr.value

    def solve16_mixed_dev(self, B, X, m=40, tol=1e-12, inner_tol=1e-6, max_outer=30, max_cycles=20, stream=None):
        """Config 5's solve A X = B (aniso_solve16_mixed_dev): 16 right-hand sides, the
        rows of B and X ((16, N) float64 CUDA tensors, original order, unit inner stride),
        fp64 refinement over fp32 inner GMRES(m), every step in the library.  Returns
        (outer refinements, inner steps, the 16 final relative residuals)."""
        import torch

        for t, name in ((B, "B"), (X, "X")):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.dim() == 2
                    and t.shape[0] == 16 and t.shape[1] == self.N and t.stride(1) == 1):
                raise ValueError(f"{name}: (16, N) float64 CUDA tensor with unit inner stride")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        outer, inner = ctypes.c_int(), ctypes.c_int()
        rel = np.zeros(16)
        _check(lib().aniso_solve16_mixed_dev(self.address, ctypes.c_void_p(B.data_ptr()), int(B.stride(0)),
                                             ctypes.c_void_p(X.data_ptr()), int(X.stride(0)), int(m), float(tol),
                                             float(inner_tol), int(max_outer), int(max_cycles), ctypes.byref(outer),
                                             ctypes.byref(inner), _dp(rel), ctypes.c_void_p(s)))
        return outer.value, inner.value, rel

    # ---- the library's own multi-GPU exchange (aniso_comm_*)
    def comm_init_rccl(self, unique_id):
        """Attach an RCCL communicator (every rank together, after set_shard)."""
        _check(lib().aniso_comm_init_rccl(self.address, bytes(unique_id)))

    def krylov_dot(self, V, w, out, stream=None):
        """out[k] = V[k] . w for the nv rows of V (aniso_krylov_dot); float64 CUDA
        tensors, V (nv, n) with unit inner stride, w (n,), out (>= nv,)."""
        import torch

        nv, n = V.shape
        _krylov_args(V, w, out, nv)
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_krylov_dot(self.address, int(n), int(nv), ctypes.c_void_p(V.data_ptr()), int(V.stride(0)),
                                      ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                      ctypes.c_void_p(s)))
        return out

    def krylov_update(self, V, c, w, out, dots=True, stream=None):
        """w -= V^T c, then out[:nv] = V w and out[nv] = w . w (dots) or out[0] = w . w
        (aniso_krylov_update)."""
        import torch

        nv, n = V.shape
        _krylov_args(V, w, out, nv + 1 if dots else 1)
        if not (c.is_cuda and c.dtype == torch.float64 and c.is_contiguous() and c.numel() >= nv):
            raise ValueError("c: contiguous float64 CUDA tensor of >= nv entries")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_krylov_update(self.address, int(n), int(nv), ctypes.c_void_p(V.data_ptr()),
                                         int(V.stride(0)), ctypes.c_void_p(c.data_ptr()),
                                         ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                         int(bool(dots)), ctypes.c_void_p(s)))
        return out

    # ---- DCGS2 Arnoldi primitives (aniso_arnoldi_*).  V: (rows, n) float64
    # CUDA tensor with unit inner stride (the Krylov vectors); w, x: n entries; state: from
    # arnoldi_state(m); status: a MappedStatus (or None); red / out: float64 CUDA tensors.
    def arnoldi_state(self, m):
        import torch

        n = ctypes.c_int64()
        _check(lib().aniso_arnoldi_state_size(int(m), ctypes.byref(n)))
        return torch.zeros(n.value, dtype=torch.float64, device="cuda")

    @staticmethod
    def _arn_v(V, rows):
        import torch

        if not (isinstance(V, torch.Tensor) and V.is_cuda and V.dtype == torch.float64 and V.dim() == 2
                and V.stride(1) == 1 and V.shape[0] >= rows):
            raise ValueError(f"V: float64 CUDA (>= {rows}, n) with unit inner stride")
        return ctypes.c_void_p(V.data_ptr()), int(V.shape[1]), int(V.stride(0))

    @staticmethod
    def _arn_t(t, n, name):
        import torch

        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
                and t.numel() >= n):
            raise ValueError(f"{name}: contiguous float64 CUDA tensor of >= {n} entries")
        return ctypes.c_void_p(t.data_ptr())

    @staticmethod
    def _arn_state(state, m):
        """the state block must hold arnoldi_state(m)'s entries: the device kernels index
        it by m's layout (H, T and R columns, g, y)"""
        n = ctypes.c_int64()
        _check(lib().aniso_arnoldi_state_size(int(m), ctypes.byref(n)))
        return Aniso._arn_t(state, n.value, f"state (arnoldi_state({int(m)}))")

    @staticmethod
    def _arn_s(stream):
        import torch

        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream if stream is None else stream)

    def arnoldi_begin(self, V, m, state, normb, rr=None, status=None, stream=None):
        pv, n, ld = self._arn_v(V, 1)
        _check(lib().aniso_arnoldi_begin(self.address, n, int(m), pv, ld, self._arn_state(state, m),
                                         None if rr is None else self._arn_t(rr, 1, "rr"), float(normb),
                                         None if status is None else status.dev, self._arn_s(stream)))

    def arnoldi_step(self, V, m, j, w, state, status=None, stream=None):
        pv, n, ld = self._arn_v(V, j + 2)
        _check(lib().aniso_arnoldi_step(self.address, n, int(m), int(j), pv, ld, self._arn_t(w, n, "w"),
                                        self._arn_state(state, m), None if status is None else status.dev,
                                        self._arn_s(stream)))

    def arnoldi_project(self, V, j, w, out, stream=None):
        pv, n, ld = self._arn_v(V, j + 1)
        _check(lib().aniso_arnoldi_project(self.address, n, int(j), pv, ld, self._arn_t(w, n, "w"),
                                           self._arn_t(out, j + 1, "out"), self._arn_s(stream)))

    def arnoldi_coef(self, m, j, state, red, stream=None):
        _check(lib().aniso_arnoldi_coef(self.address, int(m), int(j), self._arn_state(state, m),
                                        self._arn_t(red, j + 1, "red"), self._arn_s(stream)))

    def arnoldi_update(self, V, m, j, w, state, out, stream=None):
        pv, n, ld = self._arn_v(V, j + 2)
        _check(lib().aniso_arnoldi_update(self.address, n, int(m), int(j), pv, ld, self._arn_t(w, n, "w"),
                                          self._arn_state(state, m), self._arn_t(out, j + 2, "out"),
                                          self._arn_s(stream)))

    def arnoldi_column(self, m, j, state, red, status=None, stream=None):
        _check(lib().aniso_arnoldi_column(self.address, int(m), int(j), self._arn_state(state, m),
                                          self._arn_t(red, j + 2, "red"), None if status is None else status.dev,
                                          self._arn_s(stream)))

    def arnoldi_solution(self, V, m, used, state, x, stream=None):
        pv, n, ld = self._arn_v(V, max(int(used), 1))
        _check(lib().aniso_arnoldi_solution(self.address, n, int(m), int(used), pv, ld,
                                            self._arn_state(state, m), self._arn_t(x, n, "x"),
                                            self._arn_s(stream)))

    def comm_init_loopback(self):
        """Development: a loopback communicator (aniso_comm_init_loopback) to time one
        rank's schedule of an N-GPU run on one GPU; results are not the operator's."""
        _check(lib().aniso_comm_init_loopback(self.address))

    def comm_init_callbacks(self, coll):
        """Attach caller-supplied collectives (a Collectives structure; kept alive here)."""
        self._coll = coll
        _check(lib().aniso_comm_init_callbacks(self.address, ctypes.byref(coll)))

    def block_op_sharded_dev(self, which, x, y, stream=None):
        """One call of the sharded aniso.m operator: x (ks, N) tree order holds this
        rank's own range (its halo is filled here), y's owned slice receives the result."""
        import torch

        _dev_rows(x, self.ks, self.N, "x")
        _dev_rows(y, self.ks, self.N, "y")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        _check(lib().aniso_block_op_sharded_dev(self.address, int(which), ctypes.c_void_p(x.data_ptr()),
                                                int(x.stride(0)), ctypes.c_void_p(y.data_ptr()), int(y.stride(0)),
                                                ctypes.c_void_p(s)))
        return y

    def set_shard(self, rank, nranks):
        _check(lib().aniso_set_shard(self.address, int(rank), int(nranks)))

    def shard(self):
        b, e = ctypes.c_int64(), ctypes.c_int64()
        _check(lib().aniso_get_shard(self.address, ctypes.byref(b), ctypes.byref(e)))
        return b.value, e.value

    def n_owned(self):
        b, e = self.shard()
        return e - b

    def shard_cuts(self, nranks):
        """Every rank's [cuts[r], cuts[r+1]) for nranks ranks (host only, no state change)."""
        c = np.zeros(int(nranks) + 1, dtype=np.int64)
        _check(lib().aniso_shard_cuts(self.address, int(nranks), c.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return c

    def shard_exchange(self, nrhs=1):
        """The exchange plan of this handle's shard (aniso_shard_exchange), host only."""
        info = np.zeros(9, dtype=np.int64)
        _check(lib().aniso_shard_exchange(self.address, int(nrhs), info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        keys = ["root_chunk", "root_record", "halo_ranges", "halo_points", "t0_level", "t0_run", "roots_sent",
                "t0_tasks", "nranks"]
        return dict(zip(keys, (int(v) for v in info)))

    def shard_exchange_one(self):
        """The one-collective exchange of this shard (aniso_shard_exchange_one), host only."""
        info = np.zeros(5, dtype=np.int64)
        _check(lib().aniso_shard_exchange_one(self.address, info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        keys = ["ok", "own_t0_tasks", "need_nodes", "halo_ranges", "halo_points"]
        return dict(zip(keys, (int(v) for v in info)))

    def shard_upper_partials(self):
        """The upper multipoles as partial sums of this shard (aniso_shard_upper_partials), host only:
        whether the plan forms them, its tasks, records, the topmost level an M2L reads, the
        tier-0 root level, the roots the tasks cover, and the node of each record."""
        info = np.zeros(6, dtype=np.int64)
        _check(lib().aniso_shard_upper_partials(self.address, info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        keys = ["on", "tasks", "records", "top_level", "root_level", "roots"]
        d = dict(zip(keys, (int(v) for v in info)))
        nodes = np.zeros(max(d["records"], 1), dtype=np.int32)
        _check(lib().aniso_shard_upper_records(self.address, nodes.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        d["record_nodes"] = nodes[: d["records"]]
        return d

    def shard_one_halo(self):
        """(n, 2) ranges of the input the one-collective exchange fills outside the own range."""
        n = self.shard_exchange_one()["halo_ranges"]
        r = np.zeros(2 * n + 1, dtype=np.int64)
        _check(lib().aniso_shard_one_halo(self.address, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return r[:2 * n].reshape(n, 2)

    def shard_halo(self):
        """(n, 2) array of [b, e) tree-position ranges outside the own range the input must hold."""
        n = self.shard_exchange()["halo_ranges"]
        r = np.zeros(2 * n + 1, dtype=np.int64)
        _check(lib().aniso_shard_halo(self.address, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return r[: 2 * n].reshape(n, 2)

    def shard_roots(self):
        """(roots sent by this rank, all-gather slot -> node (-1 padding), roots of the tier-0 tasks run here)."""
        ex = self.shard_exchange()
        send = np.zeros(ex["roots_sent"] + 1, dtype=np.int32)
        recv = np.zeros(ex["nranks"] * ex["root_chunk"] + 1, dtype=np.int32)
        t0 = np.zeros(ex["t0_run"] + 1, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int)
        _check(lib().aniso_shard_roots(self.address, send.ctypes.data_as(ip), recv.ctypes.data_as(ip),
                                       t0.ctypes.data_as(ip)))
        return send[:-1], recv[:-1], t0[:-1]

    def tree_perm(self):
        p = np.zeros(self.N, dtype=np.int32)
        _check(lib().aniso_tree_perm(self.address, p.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return p

    def tree_size(self):
        nn, ml = ctypes.c_int(), ctypes.c_int()
        _check(lib().aniso_tree_size(self.address, ctypes.byref(nn), ctypes.byref(ml)))
        return nn.value, ml.value

    def tree_nodes(self):
        nn, _ = self.tree_size()
        ints = np.zeros((nn, 11), dtype=np.int32)
        geom = np.zeros((nn, 4))
        _check(lib().aniso_tree_nodes(self.address, ints.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _dp(geom)))
        return ints, geom

    def tree_list(self, which):
        nn, _ = self.tree_size()
        ptr = np.zeros(nn + 1, dtype=np.int64)
        _check(lib().aniso_tree_list(self.address, int(which), ptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), None))
        idx = np.zeros(int(ptr[-1]), dtype=np.int32)
        _check(lib().aniso_tree_list(self.address, int(which), ptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                     idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return ptr, idx

    def stats(self):
        s = np.zeros(40, dtype=np.int64)
        n = ctypes.c_int()
        _check(lib().aniso_stats_n(self.address, s.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(s),
                                   ctypes.byref(n)))
        keys = ["near_entries", "m2l_entries", "m2l_pairs", "leaves", "m2l_targets", "tree_nodes", "max_leaf", "N",
                "stored_near", "stored_m2l", "m2l_canon", "near_partial", "harmonic", "att_m2l_blocks",
                "hm_clusters", "hm_dual_pairs", "hm_block_reads", "f32_cache_bytes", "top_fused",
                "plan_halo_slots", "plan_max_lds_slots", "plan_block_reads", "top_recoveries",
                "near_hs_stored", "near_hs_partials", "one_exchange_applies", "mrhs_m2l_pairs",
                "top_steals", "upper_partial_applies", "near_overlap", "near_up_tier", "near_loc_entries",
                "near_corr_rows", "near_up_nodes"]
        return dict(zip(keys, (int(v) for v in s)))

    def sync(self):
        """Wait for this handle's applies and raise if any reported a device-side failure."""
        _check(lib().aniso_sync(self.address))

    def num_blocks(self):
        k = ctypes.c_int()
        _check(lib().aniso_num_blocks(self.address, ctypes.byref(k)))
        return k.value

    def set_deterministic(self, on):
        """Bitwise-reproducible block applies on / off (the clustered M2L with fixed-point
        LDS sums; ANISO_DET_PER_TARGET=1: one wave per target)."""
        _check(lib().aniso_set_deterministic(self.address, int(bool(on))))

    def set_timing(self, on):
        """0/False off, 1/True every stage, 2 the M2L and near-field spans only."""
        _check(lib().aniso_set_timing(self.address, int(on)))

    def stage_times(self):
        t = (ctypes.c_float * 8)()
        _check(lib().aniso_stage_times(self.address, t))
        return dict(zip(["exchange", "up", "m2l", "gather", "near", "down", "corr", "total"], list(t)))

    def top_trace(self):
        """Per-block timeline of the last fused top-of-tree launch (ANISO_TOP_TRACE=1):
        rows {start, waited, end (100 MHz ticks), hw id, kind (-k: up tier k, else the
        cluster id), wait tier, targets, block reads}."""
        n = ctypes.c_int64(0)
        _check(lib().aniso_top_trace(self.address, None, 0, ctypes.byref(n)))
        rec = np.zeros((n.value, 8), dtype=np.int64)
        if n.value:
            _check(lib().aniso_top_trace(self.address, rec.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n.value,
                                         ctypes.byref(n)))
        return rec

    def line_integrals(self, seg):
        seg = np.ascontiguousarray(np.asarray(seg, dtype=np.float64).reshape(-1, 4))
        out = np.zeros(seg.shape[0])
        _check(lib().aniso_line_integrals(self.address, _dp(seg), seg.shape[0], _dp(out)))
        return out


def comm_unique_id():
    """A fresh RCCL unique id (128 bytes) for aniso_comm_init_rccl."""
    b = ctypes.create_string_buffer(128)
    _check(lib().aniso_comm_unique_id(b))
    return b.raw


def memcpy(dst, src, nbytes):
    """aniso_memcpy: hipMemcpy between any two addresses (ints)."""
    _check(lib().aniso_memcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), int(nbytes)))


def block_mixes(nb, g, chi=True):
    """The (2nb-1, nb, nb) mode mixes of aniso.m forward (chi=False) / mforward (chi=True)."""
    m = np.zeros((2 * nb - 1) * nb * nb)
    _check(lib().aniso_block_mixes(int(nb), float(g), int(bool(chi)), _dp(m)))
    return m.reshape(2 * nb - 1, nb, nb)


def version():
    return lib().aniso_version().decode()
