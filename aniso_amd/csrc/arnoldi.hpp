// arnoldi.hpp -- the Arnoldi process of the device GMRES solves (aniso.m:159-173 through
// aniso_block_solve; gmres.cpp:53-169 restated) as classical Gram-Schmidt with a DELAYED
// reorthogonalisation (DCGS2) on a basis that is never rewritten.
//
// The stored vectors P = [p_0 .. p_j] (V's rows) are the raw projected residuals: each
// p_{k+1} = A q_k - Q h once orthogonalised, neither reorthogonalised nor normalised.
// The orthonormal basis is Q = P T with T upper triangular (kept in the state block):
// p_j = Q s + r q_j with s = Q^T p_j and r^2 = |p_j|^2 - |s|^2, so column j of T is
// (e_j - T s) / r.  Step j:
//
//   w  = A p_j                                   (the caller's matvec)
//   u  = P^T w                                   sweep A   k_arn_project
//   T(:, j); z = T^T u (= Q^T w); c = H s; A q_j = (w - Q c) / r (Arnoldi relation);
//   h = (z - c) / r (= Q^T A q_j); e = T (c / r + h)    k_arn_coef
//   p_{j+1} = w / r - P e  -> V[j + 1]; in the same pass u' = P^T p_{j+1}, |p_{j+1}|^2
//                                                sweep B   k_arn_update
//   s' = T^T u', r'^2 = |p_{j+1}|^2 - |s'|^2; column j of H = [h + s'; r'], its Givens
//   rotation and the residual estimate |g_{j+1}| / |b|    k_arn_column
//
// Two sweeps over the basis per step and one vector written (CGS2: three sweeps and two
// writes), and no host round trip inside a step: H, T, the rotations and g live in the
// state block; the host reads only the residual estimate.  Reductions have a fixed
// order (per-block partials, then fixed lane and row orders), so a solve is bitwise
// reproducible on a deterministic operator.  A cycle starts with V[0] = the residual
// (unnormalised) and r = its norm.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace aniso {
namespace arn {

constexpr int kThreads = 256;
constexpr int kMaxRegs = 48;  // basis rows one sweep holds in registers
constexpr int kSweepThreads = 512;  // threads per sweep block
constexpr int kParts = 256;   // blocks (partial sums per row) of a sweep: 512 x 256 measured best (tools/arnoldi_micro.hip)
constexpr int kRedRows = 16;  // rows per round of the small kernels' reductions (4 per wave)
constexpr int kUpdateVar = 0;    // k_arn_update's variant (below)
constexpr int kStageDoubles = 7000;  // LDS (55 KB) the small kernels stage T and H in

// state block (doubles) of a restart length m; M1 = m + 1
struct Layout {
    int64_t M1, Hu, R, T, s, h, e, cs, sn, g, y, sc, total;
    __host__ __device__ explicit Layout(int m) {
        M1 = m + 1;
        Hu = 0;               // Hessenberg matrix of the Arnoldi relation, M1 x m, column-major
        R = Hu + M1 * m;      // the same after the Givens rotations
        T = R + M1 * m;       // Q = P T, M1 x M1 upper triangular, column-major
        s = T + M1 * M1;      // Q^T p of the newest stored vector (M1)
        h = s + M1;           // Q^T A q_j of the current step (M1)
        e = h + M1;           // sweep B's coefficients on the stored vectors (M1)
        cs = e + M1;          // rotations (m each)
        sn = cs + m;
        g = sn + m;           // rotated right-hand side (M1)
        y = g + M1;           // the cycle's update coefficients on the stored vectors (M1)
        sc = y + M1;          // scalars (kR ...)
        total = sc + 8;
    }
};
enum { kR = 0, kInvR = 1, kNormb = 2, kRelres = 3, kSteps = 4 };

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// chunk b's contiguous element range [j0, j1)
__device__ __forceinline__ void block_range(int64_t n, int b, int64_t& j0, int64_t& j1) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t chunk = (per + 511) & ~(int64_t)511;
    j0 = min(n, (int64_t)b * chunk);
    j1 = min(n, j0 + chunk);
}

// per-block sums into part[row * gridDim.x + b] (b: the block's chunk): acc[k] is row k
// for k < used, acc[NA - 1] is row extraRow (if >= 0); wave sums by xor shuffles, then
// the 4 waves in a fixed order
template <int NA, int TB = kThreads>
__device__ __forceinline__ void block_store(const double (&acc)[NA], int used, int extraRow, double* red,
                                            double* part, int b) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NA; ++k)
        if (k < used || (k == NA - 1 && extraRow >= 0)) {
            const double v = wave_sum(acc[k]);
            if (lane == 0) red[wv * NA + k] = v;
        }
    __syncthreads();
    for (int k = threadIdx.x; k <= used; k += TB) {
        const int i = k < used ? k : NA - 1;
        const int row = k < used ? k : extraRow;
        if (row >= 0) {
            double a = red[i];
#pragma unroll
            for (int q = 1; q < TB / 64; ++q) a += red[q * NA + i];
            part[(size_t)row * gridDim.x + b] = a;
        }
    }
}

// sweep A: part[k][blk] = sum over the block's range of V[k][e] w[e], k < nv <= NV
template <int NV, int TB = kSweepThreads>
__global__ void __launch_bounds__(TB) k_arn_project(int64_t n, int nv, const double* __restrict__ V,
                                                    int64_t ldv, const double* __restrict__ w,
                                                    double* __restrict__ part) {
    __shared__ double red[(TB / 64) * NV];
    int64_t j0, j1;
    block_range(n, blockIdx.x, j0, j1);
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (int64_t e = j0 + threadIdx.x; e < j1; e += TB) {
        double v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < nv) v[k] = V[(size_t)k * ldv + e];
        const double we = w[e];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < nv) acc[k] = __builtin_fma(v[k], we, acc[k]);
    }
    block_store<NV, TB>(acc, nv, -1, red, part, blockIdx.x);
}

// sweep B for nv = j + 1 <= NV stored rows: p = w inv_r - sum_k e_k V_k -> V[nv]; the
// partials of V_k . p (rows k < nv) and p . p (row nv)
// VAR (development variants, tools/arnoldi_micro.hip, neither faster): bit 0 chunks in
// reverse launch order (the chunks sweep A read last first, for Infinity-Cache hits);
// bit 2 non-temporal stores of p.  The one store stream costs ~50 us at 1M x 5 among the
// nv + 1 read streams (4.7-4.9 against 5.9-6.0 TB/s without it; row padding, store
// placement and store kind do not change it: profiles/r05h-j_micro.log)
template <int NV, int VAR = kUpdateVar, int TB = kSweepThreads>
__global__ void __launch_bounds__(TB) k_arn_update(int64_t n, int nv, double* __restrict__ V, int64_t ldv,
                                                         const double* __restrict__ w,
                                                         const double* __restrict__ st, int m,
                                                         double* __restrict__ part) {
    constexpr int NA = NV + 1;
    __shared__ double red[(TB / 64) * NA];
    __shared__ double cf[NV + 1];  // -e[0 .. nv), inv_r
    const Layout L(m);
    for (int k = threadIdx.x; k < NV; k += TB) cf[k] = k < nv ? -st[L.e + k] : 0.0;
    if (threadIdx.x == 0) cf[NV] = st[L.sc + kInvR];
    __syncthreads();
    const double ir = cf[NV];
    const int b = (VAR & 1) ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
    int64_t j0, j1;
    block_range(n, b, j0, j1);
    double acc[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) acc[k] = 0.0;
    double* __restrict__ Vn = V + (size_t)nv * ldv;
    // p of the previous element is stored after this element's loads are issued: vmcnt
    // counts stores with loads (MI355X_MICROARCH.md, s_waitcnt), so a store issued before
    // them would hold the later load waits to its acknowledgement
    // (unconditional: the first iteration stores 0 into its own element's slot, which the
    // second overwrites -- a store under a branch would again drain with the loads)
    double pPrev = 0.0;
    int64_t ePrev = j0 + threadIdx.x;
    for (int64_t e = j0 + threadIdx.x; e < j1; e += TB) {
        // rows past nv re-read row nv - 1 (an L1 hit) with a zero coefficient: no branch
        // per row, so the compiler can count the loads in its vmcnt waits instead of
        // draining the store below with them
        double v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = V[(size_t)(k < nv ? k : nv - 1) * ldv + e];
        const double we = w[e];
        // the loads above are issued before the store below, and cf is re-read from LDS
        // per element instead of held in NV registers
        asm volatile("" ::: "memory");
        if constexpr ((VAR & 4) != 0) __builtin_nontemporal_store(pPrev, Vn + ePrev);
        else Vn[ePrev] = pPrev;
        double p = we * ir;
#pragma unroll
        for (int k = 0; k < NV; ++k) p = __builtin_fma(cf[k], v[k], p);
        pPrev = p;
        ePrev = e;
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = __builtin_fma(v[k], p, acc[k]);  // rows >= nv: not stored
        acc[NA - 1] = __builtin_fma(p, p, acc[NA - 1]);
    }
    if (ePrev < j1) Vn[ePrev] = pPrev;
    block_store<NA, TB>(acc, nv, nv, red, part, b);
}

// sweep B beyond kMaxRegs rows, first half: p -> V[nv] (one read of V, no register
// limit); the partials then come from k_arn_project over V[0 .. nv] with w = p (a
// second read of V, only past kMaxRegs rows)
__global__ void __launch_bounds__(kThreads) k_arn_update_wide(int64_t n, int nv, double* __restrict__ V, int64_t ldv,
                                                              const double* __restrict__ w,
                                                              const double* __restrict__ st, int m) {
    extern __shared__ double cw[];  // -e[0 .. nv)
    const Layout L(m);
    for (int k = threadIdx.x; k < nv; k += kThreads) cw[k] = -st[L.e + k];
    __syncthreads();
    const double ir = st[L.sc + kInvR];
    const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (e >= n) return;
    double p = w[e] * ir;
    for (int k = 0; k < nv; ++k) p = __builtin_fma(cw[k], V[(size_t)k * ldv + e], p);
    V[(size_t)nv * ldv + e] = p;
}

// ---- the small kernels (one block per column: the one-vector solves launch one, the
// 16-column solve of config 5 one per column, blockIdx.x = the column).  Row sums of
// partials part[k * rs + b], b < P = kParts (rs = kParts for one column, 16 kParts for
// 16 interleaved columns), in a fixed order: lane l sums its kParts / 64 consecutive
// partials, the 64 lane sums go through LDS, thread k adds them in lane order.  P = 1:
// the values themselves (a caller's all-reduced sums, one column).  scratch: kRedRows
// x 64 doubles of LDS; out: LDS.
__device__ __forceinline__ void reduce_rows(const double* __restrict__ part, int P, int64_t rs, int rows, double* out,
                                            double* scratch) {
    if (P == 1) {
        for (int k = threadIdx.x; k < rows; k += kThreads) out[k] = part[k];
        __syncthreads();
        return;
    }
    // P == kParts: lane l sums partials [l * kPer, (l + 1) * kPer) of a row, every load of
    // a wave's four rows in flight at once
    constexpr int kPer = kParts / 64;
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k0 = 0; k0 < rows; k0 += kRedRows) {
        const int nr = rows - k0 < kRedRows ? rows - k0 : kRedRows;
        d2 v[4][kPer / 2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = wv + 4 * q;
            const d2* pr = (const d2*)(part + (size_t)(k0 + (r < nr ? r : 0)) * rs + (size_t)lane * kPer);
#pragma unroll
            for (int b = 0; b < kPer / 2; ++b) v[q][b] = pr[b];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double a = 0.0;
#pragma unroll
            for (int b = 0; b < kPer / 2; ++b) a += v[q][b].x + v[q][b].y;
            if (wv + 4 * q < nr) scratch[(wv + 4 * q) * 64 + lane] = a;
        }
        __syncthreads();
        for (int r = threadIdx.x; r < nr; r += kThreads) {  // fast_rows_finish's order
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
            for (int l = 0; l < 64; l += 4) {
                a0 += scratch[r * 64 + l];
                a1 += scratch[r * 64 + l + 1];
                a2 += scratch[r * 64 + l + 2];
                a3 += scratch[r * 64 + l + 3];
            }
            out[k0 + r] = (a0 + a1) + (a2 + a3);
        }
        __syncthreads();
    }
}

// y[0 .. rows) = A x for a column-major A (rows x cols at lda) restricted to its band
// k >= i - lo (Hessenberg: lo = 1; upper triangular: lo = 0), x in LDS; thread i
// accumulates over the columns in order
__device__ __forceinline__ void band_matvec(const double* __restrict__ A, int64_t lda, int rows, int cols, int lo,
                                            const double* x, double* y) {
    for (int i = threadIdx.x; i < rows; i += kThreads) {
        double a = 0.0;
        const int k0 = i - lo > 0 ? i - lo : 0;
#pragma unroll 8
        for (int k = k0; k < cols; ++k) a = __builtin_fma(A[i + k * lda], x[k], a);
        y[i] = a;
    }
}

// y[0 .. n) = T^T x for the upper-triangular T (column i: rows 0 .. i), x in LDS
__device__ __forceinline__ void triT_matvec(const double* __restrict__ T, int64_t ldt, int n, const double* x,
                                            double* y) {
    for (int i = threadIdx.x; i < n; i += kThreads) {
        double a = 0.0;
        const double* Ti = T + (size_t)i * ldt;
#pragma unroll 8
        for (int k = 0; k <= i; ++k) a = __builtin_fma(Ti[k], x[k], a);
        y[i] = a;
    }
}

// the leading rows x cols block of a column-major matrix (lda) into LDS, dense at ld
// rows; every load in flight before the stores
__device__ __forceinline__ void stage(const double* __restrict__ A, int64_t lda, int rows, int cols, double* S) {
    const int nn = rows * cols;
    for (int f0 = 0; f0 < nn; f0 += 8 * kThreads) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int f = f0 + q * kThreads + threadIdx.x;
            if (f < nn) v[q] = A[(f % rows) + (int64_t)(f / rows) * lda];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int f = f0 + q * kThreads + threadIdx.x;
            if (f < nn) S[f] = v[q];
        }
    }
}

// ---- one-round fast paths of the small kernels (rows <= kFast): every global load of
// the kernel (partials, the staged matrices, vectors) is issued before the first is
// used.  Wave wv owns partial rows wv + 4q and matrix columns wv + 4q (q < 16); a
// lane reads kParts / 64 consecutive partials of a row, or one matrix row.
constexpr int kFast = 64;
typedef double d2f __attribute__((ext_vector_type(2)));

struct FastRows {
    d2f v[16][kParts / 128];
};

__device__ __forceinline__ void fast_rows_load(const double* __restrict__ part, int P, int64_t rs, int rows,
                                               FastRows& fr) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (P == 1) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int r = wv + 4 * q;
        if (r < rows) {
            const d2f* pr = (const d2f*)(part + (size_t)r * rs + (size_t)lane * (kParts / 64));
#pragma unroll
            for (int b = 0; b < kParts / 128; ++b) fr.v[q][b] = pr[b];
        }
    }
}

// the rows' sums into out (LDS) in a fixed order; scratch: kFast x 64 doubles
__device__ __forceinline__ void fast_rows_finish(const double* __restrict__ part, int P, int rows, const FastRows& fr,
                                                 double* scratch, double* out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (P == 1) {
        for (int k = threadIdx.x; k < rows; k += kThreads) out[k] = part[k];
        return;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int r = wv + 4 * q;
        if (r < rows) {
            double a = 0.0;
#pragma unroll
            for (int b = 0; b < kParts / 128; ++b) a += fr.v[q][b].x + fr.v[q][b].y;
            scratch[r * 64 + lane] = a;
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < rows; r += kThreads) {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
        for (int l = 0; l < 64; l += 4) {
            a0 += scratch[r * 64 + l];
            a1 += scratch[r * 64 + l + 1];
            a2 += scratch[r * 64 + l + 2];
            a3 += scratch[r * 64 + l + 3];
        }
        out[r] = (a0 + a1) + (a2 + a3);
    }
}

// columns [0, cols) of a column-major matrix (rows <= 64 at lda) into registers, then LDS
// (dense at ld rows)
struct FastCols {
    double v[16];
};

__device__ __forceinline__ void fast_cols_load(const double* __restrict__ A, int64_t lda, int rows, int cols,
                                               FastCols& fc) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int c = wv + 4 * q;
        if (c < cols && lane < rows) fc.v[q] = A[lane + (int64_t)c * lda];
    }
}

__device__ __forceinline__ void fast_cols_store(const FastCols& fc, int rows, int cols, double* S) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int c = wv + 4 * q;
        if (c < cols && lane < rows) S[c * rows + lane] = fc.v[q];
    }
}

// k_arn_coef for j + 1 <= kFast.  LDS: scratch (kFast x 64) | u s tc c d (5 x 64) | T (n1 x j) | H (n1 x j)
__device__ __forceinline__ void coef_fast(int m, int j, double* __restrict__ st, const double* __restrict__ part,
                                          int P, int64_t rs, double* sm) {
    const int n1 = j + 1;
    double* scratch = sm;
    double *u = sm + kFast * 64, *s = u + kFast, *tc = s + kFast, *c = tc + kFast, *d = c + kFast;
    double* Ts = d + kFast;
    double* Hs = Ts + n1 * j;
    const Layout L(m);
    double* Tg = st + L.T;
    FastRows fr;
    FastCols ft, fh;
    fast_rows_load(part, P, rs, n1, fr);
    fast_cols_load(Tg, L.M1, n1, j, ft);
    fast_cols_load(st + L.Hu, L.M1, n1, j, fh);
    const double sv = threadIdx.x < j ? st[L.s + threadIdx.x] : 0.0;
    const double r = st[L.sc + kR];
    fast_cols_store(ft, n1, j, Ts);
    fast_cols_store(fh, n1, j, Hs);
    if (threadIdx.x < j) s[threadIdx.x] = sv;
    fast_rows_finish(part, P, n1, fr, scratch, u);
    __syncthreads();
    const double ir = r > 0.0 ? 1.0 / r : 0.0;  // r = 0: a finished column, q_j = 0 (no NaN)
    band_matvec(Ts, n1, j, j, 0, s, tc);  // T s
    band_matvec(Hs, n1, n1, j, 1, s, c);  // H s
    __syncthreads();
    for (int i = threadIdx.x; i <= j; i += kThreads) {
        const double t = i < j ? -tc[i] * ir : ir;  // column j of T: (e_j - T s) / r
        tc[i] = t;
        Tg[i + (size_t)j * L.M1] = t;
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= j; i += kThreads) {  // z = T^T u, h, d
        double a = 0.0;
        if (i < j) {
            for (int k = 0; k <= i; ++k) a = __builtin_fma(Ts[i * n1 + k], u[k], a);
        } else {
            for (int k = 0; k <= j; ++k) a = __builtin_fma(tc[k], u[k], a);
        }
        const double hi = (a - c[i]) * ir;
        st[L.h + i] = hi;
        d[i] = __builtin_fma(c[i], ir, hi);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= j; i += kThreads) {  // e = T d
        double a = 0.0;
        for (int k = i; k < j; ++k) a = __builtin_fma(Ts[k * n1 + i], d[k], a);
        st[L.e + i] = __builtin_fma(tc[i], d[j], a);
    }
    if (threadIdx.x == 0) st[L.sc + kInvR] = ir;
}

inline __host__ __device__ size_t coef_fast_lds(int j) { return ((size_t)kFast * 69 + (size_t)2 * (j + 1) * j) * 8; }

// k_arn_column for j + 2 <= kFast.  LDS: scratch (kFast x 64) | u' s' col cs sn h (6 x 64) | T (n1 x n1)
__device__ __forceinline__ void column_fast(int m, int j, double* __restrict__ st, const double* __restrict__ part,
                                            int P, int64_t rs, double* __restrict__ status, double* sm) {
    const int n1 = j + 1;
    double* scratch = sm;
    double *up = sm + kFast * 64, *sp = up + kFast, *col = sp + kFast, *csl = col + kFast, *snl = csl + kFast,
           *hl = snl + kFast;
    double* Ts = hl + kFast;
    __shared__ double ssum;
    const Layout L(m);
    FastRows fr;
    FastCols ft;
    fast_rows_load(part, P, rs, j + 2, fr);
    fast_cols_load(st + L.T, L.M1, n1, n1, ft);
    const int t = threadIdx.x;
    const double cv = t < j ? st[L.cs + t] : 0.0, sv = t < j ? st[L.sn + t] : 0.0;
    const double hv = t <= j ? st[L.h + t] : 0.0;
    const double gj = st[L.g + j], normb = st[L.sc + kNormb];
    fast_cols_store(ft, n1, n1, Ts);
    if (t < j) {
        csl[t] = cv;
        snl[t] = sv;
    }
    if (t <= j) hl[t] = hv;
    fast_rows_finish(part, P, j + 2, fr, scratch, up);
    __syncthreads();
    for (int i = t; i <= j; i += kThreads) {  // s' = T^T u' = Q^T p
        double a = 0.0;
        for (int k = 0; k <= i; ++k) a = __builtin_fma(Ts[i * n1 + k], up[k], a);
        sp[i] = a;
    }
    __syncthreads();
    if (t < 64) {
        double ss = 0.0;
        for (int k = t; k <= j; k += 64) ss = __builtin_fma(sp[k], sp[k], ss);
        ss = wave_sum(ss);
        if (t == 0) ssum = ss;
    }
    double* Hu = st + L.Hu + (size_t)j * L.M1;
    double* R = st + L.R + (size_t)j * L.M1;
    for (int i = t; i <= j; i += kThreads) {
        const double v = hl[i] + sp[i];
        Hu[i] = v;
        col[i] = v;
        st[L.s + i] = sp[i];
    }
    __syncthreads();
    if (t == 0) {
        const double a2 = up[j + 1] - ssum;
        const double r = sqrt(a2 > 0.0 ? a2 : 0.0);
        Hu[j + 1] = r;
        st[L.sc + kR] = r;
        double a = col[0];
        for (int k = 0; k < j; ++k) {  // the previous rotations, R[k + 1] carried in a register
            const double b = col[k + 1];
            col[k] = csl[k] * a + snl[k] * b;
            a = -snl[k] * a + csl[k] * b;
        }
        const double den = hypot(a, r);
        const double c = den == 0.0 ? 1.0 : a / den;
        const double sn = den == 0.0 ? 0.0 : r / den;
        st[L.cs + j] = c;
        st[L.sn + j] = sn;
        col[j] = den;
        col[j + 1] = 0.0;
        st[L.g + j + 1] = -sn * gj;
        st[L.g + j] = c * gj;
        const double rel = fabs(sn * gj) / normb;
        st[L.sc + kRelres] = rel;
        st[L.sc + kSteps] = j + 1;
        if (status) {
            status[0] = rel;
            status[1] = r;
            status[2] = j + 1;
        }
    }
    __syncthreads();
    for (int i = t; i <= j + 1; i += kThreads) R[i] = col[i];
}

inline __host__ __device__ size_t column_fast_lds(int j) { return ((size_t)kFast * 70 + (size_t)(j + 1) * (j + 1)) * 8; }

// Column c = blockIdx.x of a solve with several interleaved columns: its state block at
// st + c * sts, its partials at part + c * pc (row stride rs), its status at status +
// c * ss; one column: sts = pc = 0, rs = kParts.
struct ColArgs {
    int64_t sts, pc, rs;
    int ss;
};
constexpr ColArgs kOneCol{0, 0, kParts, 0};

// cycle start: V[0] holds the residual r; rr = |r|^2 (P partials, or P = 1: reduced);
// normb: |b| (normbv: per column, else the scalar); status (may be null): {|r| / normb, |r|, 0}
__global__ void __launch_bounds__(kThreads) k_arn_begin(int m, double* __restrict__ st, const double* __restrict__ rr,
                                                        int P, double normb, double* __restrict__ status,
                                                        ColArgs ca = kOneCol, const double* __restrict__ normbv = nullptr) {
    __shared__ double scratch[kRedRows * 64];
    __shared__ double a[1];
    const int c = blockIdx.x;
    st += c * ca.sts;
    rr += P == 1 ? c : c * ca.pc;
    if (status) status += c * ca.ss;
    if (normbv) normb = normbv[c];
    const Layout L(m);
    reduce_rows(rr, P, ca.rs, 1, a, scratch);
    const double r = sqrt(a[0] > 0.0 ? a[0] : 0.0);
    for (int k = threadIdx.x; k < L.M1; k += kThreads) st[L.g + k] = k == 0 ? r : 0.0;
    if (threadIdx.x == 0) {
        st[L.sc + kR] = r;
        st[L.sc + kNormb] = normb;
        st[L.sc + kRelres] = r / normb;
        st[L.sc + kSteps] = 0;
        if (status) {
            status[0] = r / normb;
            status[1] = r;
            status[2] = 0;
        }
    }
}

// coefficients of step j from sweep A's sums u = P^T w (rows 0 .. j), for j + 1 > kFast:
// T (columns 0 .. j - 1) and H read from the state block (2 (j + 1) j doubles exceed the
// LDS stage, kStageDoubles, for every such j)
__device__ __forceinline__ void coef_body(int m, int j, double* __restrict__ st, double* sm) {
    const int n1 = j + 1;
    double *u = sm, *s = u + n1, *tc = s + n1, *z = tc + n1, *c = z + n1, *d = c + n1;
    (void)z;
    const Layout L(m);
    double* Tg = st + L.T;
    const double* T = Tg;
    const double* H = st + L.Hu;
    const int64_t ldt = L.M1, ldh = L.M1;
    const double r = st[L.sc + kR];
    const double ir = r > 0.0 ? 1.0 / r : 0.0;
    // column j of T: (e_j - T s) / r
    band_matvec(T, ldt, j, j, 0, s, tc);
    // c = H s
    band_matvec(H, ldh, n1, j, 1, s, c);
    __syncthreads();
    for (int i = threadIdx.x; i <= j; i += kThreads) {
        const double t = i < j ? -tc[i] * ir : ir;
        tc[i] = t;
        Tg[i + (size_t)j * L.M1] = t;
    }
    __syncthreads();
    // z = T^T u (column j from tc)
    for (int i = threadIdx.x; i <= j; i += kThreads) {
        double a = 0.0;
        if (i < j) {
            const double* Ti = T + (size_t)i * ldt;
#pragma unroll 8
            for (int k = 0; k <= i; ++k) a = __builtin_fma(Ti[k], u[k], a);
        } else {
            for (int k = 0; k <= j; ++k) a = __builtin_fma(tc[k], u[k], a);
        }
        const double hi = (a - c[i]) * ir;
        st[L.h + i] = hi;
        d[i] = __builtin_fma(c[i], ir, hi);
    }
    __syncthreads();
    // e = T d (upper triangular: row i, columns i .. j; column j from tc)
    for (int i = threadIdx.x; i <= j; i += kThreads) {
        double a = 0.0;
#pragma unroll 8
        for (int k = i; k < j; ++k) a = __builtin_fma(T[i + (size_t)k * ldt], d[k], a);
        st[L.e + i] = __builtin_fma(tc[i], d[j], a);
    }
    if (threadIdx.x == 0) st[L.sc + kInvR] = ir;
}

__global__ void __launch_bounds__(kThreads) k_arn_coef(int m, int j, double* __restrict__ st,
                                                       const double* __restrict__ part, int P, ColArgs ca = kOneCol) {
    extern __shared__ double sm[];  // fast path: coef_fast's layout; else u, s, tcol, z, c, d: 6 (j + 1)
    __shared__ double scratch[kRedRows * 64];
    st += blockIdx.x * ca.sts;
    part += P == 1 ? 0 : blockIdx.x * ca.pc;
    if (j + 1 <= kFast) {
        coef_fast(m, j, st, part, P, ca.rs, sm);
        return;
    }
    const Layout L(m);
    reduce_rows(part, P, ca.rs, j + 1, sm, scratch);
    for (int k = threadIdx.x; k < j; k += kThreads) sm[j + 1 + k] = st[L.s + k];
    __syncthreads();
    coef_body(m, j, st, sm);
}

inline __host__ __device__ bool column_staged(int j) {
    return (int64_t)(j + 1) * (j + 1) + 3 * (j + 2) + 2 * j <= kStageDoubles;
}

// column j of H from sweep B's sums (rows 0 .. j: u' = P^T p, row j + 1: |p|^2), the
// Givens rotations (gmres.cpp:131-150) and the residual estimate; status (may be
// null): {relres, r', steps}
__global__ void __launch_bounds__(kThreads) k_arn_column(int m, int j, double* __restrict__ st,
                                                         const double* __restrict__ part, int P,
                                                         double* __restrict__ status, ColArgs ca = kOneCol) {
    extern __shared__ double sm[];  // fast path: column_fast's layout; else u'[0 .. j + 1] | s' | col[0 .. j + 1] | cs | sn
    __shared__ double scratch[kRedRows * 64];
    __shared__ double ssum;
    st += blockIdx.x * ca.sts;
    part += P == 1 ? 0 : blockIdx.x * ca.pc;
    if (status) status += blockIdx.x * ca.ss;
    if (j + 2 <= kFast) {
        column_fast(m, j, st, part, P, ca.rs, status, sm);
        return;
    }
    double* up = sm;
    double* sp = up + (j + 2);
    double* col = sp + (j + 1);
    double* csl = col + (j + 2);
    double* snl = csl + j;
    const Layout L(m);
    reduce_rows(part, P, ca.rs, j + 2, up, scratch);
    for (int k = threadIdx.x; k < j; k += kThreads) {
        csl[k] = st[L.cs + k];
        snl[k] = st[L.sn + k];
    }
    // s' = T^T u' = Q^T p (T staged in LDS where it fits)
    if (column_staged(j)) {
        double* Ts = snl + j;
        stage(st + L.T, L.M1, j + 1, j + 1, Ts);
        __syncthreads();
        triT_matvec(Ts, j + 1, j + 1, up, sp);
    } else {
        triT_matvec(st + L.T, L.M1, j + 1, up, sp);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        double ss = 0.0;
        for (int k = threadIdx.x; k <= j; k += 64) ss = __builtin_fma(sp[k], sp[k], ss);
        ss = wave_sum(ss);
        if (threadIdx.x == 0) ssum = ss;
    }
    double* Hu = st + L.Hu + (size_t)j * L.M1;
    double* R = st + L.R + (size_t)j * L.M1;
    for (int i = threadIdx.x; i <= j; i += kThreads) {
        const double v = st[L.h + i] + sp[i];
        Hu[i] = v;
        col[i] = v;
        st[L.s + i] = sp[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double a2 = up[j + 1] - ssum;
        const double r = sqrt(a2 > 0.0 ? a2 : 0.0);
        Hu[j + 1] = r;
        st[L.sc + kR] = r;
        // the previous rotations, R[k + 1] carried in a register
        double a = col[0];
        for (int k = 0; k < j; ++k) {
            const double b = col[k + 1];
            col[k] = csl[k] * a + snl[k] * b;
            a = -snl[k] * a + csl[k] * b;
        }
        const double den = hypot(a, r);
        const double c = den == 0.0 ? 1.0 : a / den;
        const double sn = den == 0.0 ? 0.0 : r / den;
        st[L.cs + j] = c;
        st[L.sn + j] = sn;
        col[j] = den;
        col[j + 1] = 0.0;
        double* g = st + L.g;
        const double gj = g[j];
        g[j + 1] = -sn * gj;
        g[j] = c * gj;
        const double rel = fabs(sn * gj) / st[L.sc + kNormb];
        st[L.sc + kRelres] = rel;
        st[L.sc + kSteps] = j + 1;
        if (status) {
            status[0] = rel;
            status[1] = r;
            status[2] = j + 1;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= j + 1; i += kThreads) R[i] = col[i];
}

inline __host__ __device__ bool solve_staged(int used) { return (int64_t)used * (used + 2) <= kStageDoubles; }

// the cycle's update coefficients on the stored vectors: R yh = g over the used columns
// (back substitution column by column), then y = T yh
__global__ void __launch_bounds__(kThreads) k_arn_solve(int m, int used, double* __restrict__ st, int64_t sts = 0) {
    extern __shared__ double t[];  // t[0 .. used), yh[0 .. used), staged R
    st += blockIdx.x * sts;
    double* yh = t + used;
    double* Rs = yh + used;
    const Layout L(m);
    const bool staged = solve_staged(used);
    if (staged) stage(st + L.R, L.M1, used, used, Rs);
    const double* R = staged ? Rs : st + L.R;
    const int64_t ldr = staged ? used : L.M1;
    for (int i = threadIdx.x; i < used; i += kThreads) t[i] = st[L.g + i];
    __syncthreads();
    for (int k = used - 1; k >= 0; --k) {
        if (threadIdx.x == 0) {
            const double dk = R[k + (size_t)k * ldr];
            yh[k] = dk != 0.0 ? t[k] / dk : 0.0;
        }
        __syncthreads();
        const double y = yh[k];
        for (int i = threadIdx.x; i < k; i += kThreads) t[i] = __builtin_fma(-R[i + (size_t)k * ldr], y, t[i]);
        __syncthreads();
    }
    band_matvec(st + L.T, L.M1, used, used, 0, yh, st + L.y);
}

// x[e] += sum_{k < nv} y[k] V[k][e] (y: the state block's update coefficients)
__global__ void __launch_bounds__(kThreads) k_arn_axpy(int64_t n, int nv, const double* __restrict__ V, int64_t ldv,
                                                       const double* __restrict__ y, double* __restrict__ x) {
    extern __shared__ double ys[];
    for (int k = threadIdx.x; k < nv; k += kThreads) ys[k] = y[k];
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (e >= n) return;
    double a = x[e];
    for (int k = 0; k < nv; ++k) a = __builtin_fma(ys[k], V[(size_t)k * ldv + e], a);
    x[e] = a;
}

// row sums of partials (P columns) into out (device): the multi-rank path's local sums
__global__ void __launch_bounds__(kThreads) k_arn_rows(const double* __restrict__ part, int P, int rows,
                                                       double* __restrict__ out) {
    __shared__ double scratch[kRedRows * 64];
    extern __shared__ double o[];
    reduce_rows(part, P, kParts, rows, o, scratch);
    for (int k = threadIdx.x; k < rows; k += kThreads) out[k] = o[k];
}

// ---- host launchers
template <typename F>
inline void nv_dispatch(int nv, F&& f) {
    if (nv <= 8) f(std::integral_constant<int, 8>{});
    else if (nv <= 16) f(std::integral_constant<int, 16>{});
    else if (nv <= 24) f(std::integral_constant<int, 24>{});
    else if (nv <= 32) f(std::integral_constant<int, 32>{});
    else if (nv <= 40) f(std::integral_constant<int, 40>{});
    else f(std::integral_constant<int, kMaxRegs>{});
}

// part[k * kParts + b] (k < nv): sweep A, in groups of kMaxRegs rows (w re-read per group)
template <int TB = kSweepThreads, int PP = kParts>
inline void launch_project(int64_t n, int nv, const double* V, int64_t ldv, const double* w, double* part,
                           hipStream_t s) {
    for (int k0 = 0; k0 < nv; k0 += kMaxRegs) {
        const int g = nv - k0 < kMaxRegs ? nv - k0 : kMaxRegs;
        const double* Vg = V + (size_t)k0 * ldv;
        double* pg = part + (size_t)k0 * PP;
        nv_dispatch(g, [&](auto c) {
            k_arn_project<decltype(c)::value, TB><<<PP, TB, 0, s>>>(n, g, Vg, ldv, w, pg);
        });
    }
}

// sweep B of step j (nv = j + 1 stored rows): V[nv] written, part rows 0 .. nv
template <int VAR = kUpdateVar, int TB = kSweepThreads, int PP = kParts>
inline void launch_update(int64_t n, int nv, double* V, int64_t ldv, const double* w, const double* st, int m,
                          double* part, hipStream_t s) {
    if (nv <= kMaxRegs) {
        nv_dispatch(nv, [&](auto c) {
            k_arn_update<decltype(c)::value, VAR, TB><<<PP, TB, 0, s>>>(n, nv, V, ldv, w, st, m, part);
        });
        return;
    }
    k_arn_update_wide<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, (size_t)nv * sizeof(double), s>>>(
        n, nv, V, ldv, w, st, m);
    launch_project<TB, PP>(n, nv + 1, V, ldv, V + (size_t)nv * ldv, part, s);
}

inline size_t coef_lds(int j) {
    if (j + 1 <= kFast) return coef_fast_lds(j);
    return (size_t)6 * (j + 1) * sizeof(double);
}
inline size_t column_lds(int j) {
    if (j + 2 <= kFast) return column_fast_lds(j);
    return ((size_t)(3 * (j + 2) + 2 * j) + (column_staged(j) ? (size_t)(j + 1) * (j + 1) : 0)) * sizeof(double);
}
inline size_t solve_lds(int used) { return ((size_t)2 * used + (solve_staged(used) ? (size_t)used * used : 0)) * sizeof(double); }

}  // namespace arn
}  // namespace aniso
