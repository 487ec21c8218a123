// arnoldi16.hpp -- config 5's inner Krylov process (SURVEY.md §8(d) config 5 over
// main.cpp:121-141 / gmres.cpp:53-169): 16 independent GMRES right-hand sides advanced
// in lockstep on an fp32 basis, the DCGS2 Arnoldi of arnoldi.hpp per
// column.  The vectors are the 16-right-hand-side operators' layout: N x 16 point-major
// in tree order (aniso_forward_f32_dev), so column c of a basis row is every 16th
// element from c.  The sweeps read the fp32 rows and the fp32 operator output and
// accumulate in fp64; the stored direction p_{j+1} is rounded to fp32 and its inner
// products are taken with the rounded values, so T (Q = P T) describes the stored
// basis exactly.  The small per-column kernels are arnoldi.hpp's, one block per column
// (ColArgs).  Partials: part[(row * 16 + c) * kParts + b].
#pragma once

#include "arnoldi.hpp"

namespace aniso {
namespace arn16 {

constexpr int KC = 16;               // interleaved columns (right-hand sides)
constexpr int kT = 512;              // threads per sweep block (a multiple of KC)
constexpr int kParts = arn::kParts;  // blocks per sweep
constexpr int kMaxRows = 48;         // basis rows one sweep holds in registers
constexpr arn::ColArgs kCols{0, kParts, (int64_t)KC * kParts, 4};  // + sts at the launch

// per-block sums of acc[k] (k < used, and acc[NA - 1] as row extraRow if >= 0) over the
// block's threads of each column: xor shuffles over lanes 16 and 32 apart (same
// column), then the kT / 64 waves in a fixed order
template <int NA>
__device__ __forceinline__ void block_store16(const double (&acc)[NA], int used, int extraRow, double* red,
                                              double* part, int b) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NA; ++k)
        if (k < used || (k == NA - 1 && extraRow >= 0)) {
            double v = acc[k];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < KC) red[(wv * NA + k) * KC + lane] = v;
        }
    __syncthreads();
    for (int f = threadIdx.x; f < (used + 1) * KC; f += kT) {
        const int k = f / KC, c = f % KC;
        const int i = k < used ? k : NA - 1;
        const int row = k < used ? k : extraRow;
        if (row >= 0) {
            double a = red[i * KC + c];
#pragma unroll
            for (int q = 1; q < kT / 64; ++q) a += red[(q * NA + i) * KC + c];
            part[((size_t)row * KC + c) * gridDim.x + b] = a;
        }
    }
}

// sweep A: partials of V_k[:, c] . w[:, c], k < nv <= NV (n16 = 16 N elements)
template <int NV>
__global__ void __launch_bounds__(kT) k16_project(int64_t n16, int nv, const float* __restrict__ V, int64_t ldv,
                                                  const float* __restrict__ w, double* __restrict__ part) {
    __shared__ double red[(kT / 64) * NV * KC];
    int64_t j0, j1;
    arn::block_range(n16, blockIdx.x, j0, j1);
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (int64_t e = j0 + threadIdx.x; e < j1; e += kT) {
        float v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < nv) v[k] = V[(size_t)k * ldv + e];
        const double we = w[e];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < nv) acc[k] = __builtin_fma((double)v[k], we, acc[k]);
    }
    block_store16<NV>(acc, nv, -1, red, part, blockIdx.x);
}

// sweep B for nv = j + 1 stored rows: p = w inv_r - sum_k e_k V_k per column, stored
// (rounded to fp32) as V[nv]; the partials of V_k . p (k < nv) and p . p (row nv) with
// the rounded p.  st: the 16 state blocks, sts apart.
template <int NV>
__global__ void __launch_bounds__(kT) k16_update(int64_t n16, int nv, float* __restrict__ V, int64_t ldv,
                                                 const float* __restrict__ w, const double* __restrict__ st,
                                                 int64_t sts, int m, double* __restrict__ part) {
    constexpr int NA = NV + 1;
    __shared__ double red[(kT / 64) * NA * KC];
    __shared__ double cf[(NV + 1) * KC];  // -e_c[0 .. nv) rows, inv_r_c
    const arn::Layout L(m);
    for (int f = threadIdx.x; f < (NV + 1) * KC; f += kT) {
        const int k = f / KC, c = f % KC;
        const double* sc = st + c * sts;
        cf[f] = k < NV ? (k < nv ? -sc[L.e + k] : 0.0) : sc[L.sc + arn::kInvR];
    }
    __syncthreads();
    const int c = threadIdx.x % KC;
    const double ir = cf[NV * KC + c];
    int64_t j0, j1;
    arn::block_range(n16, blockIdx.x, j0, j1);
    double acc[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) acc[k] = 0.0;
    float* __restrict__ Vn = V + (size_t)nv * ldv;
    for (int64_t e = j0 + threadIdx.x; e < j1; e += kT) {
        float v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = V[(size_t)(k < nv ? k : nv - 1) * ldv + e];
        double p = (double)w[e] * ir;
#pragma unroll
        for (int k = 0; k < NV; ++k) p = __builtin_fma(cf[k * KC + c], (double)v[k], p);
        const float pf = (float)p;
        Vn[e] = pf;
        const double pr = (double)pf;
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = __builtin_fma((double)v[k], pr, acc[k]);  // rows >= nv: not stored
        acc[NA - 1] = __builtin_fma(pr, pr, acc[NA - 1]);
    }
    block_store16<NA>(acc, nv, nv, red, part, blockIdx.x);
}

// out = a - b (b may be null) per element, fp64 and/or rounded to fp32 (either output
// may be null), and the partials of |out|^2 per column (of the fp32 value when vf is
// written: the norm of the stored vector); part[c * kParts + b]
template <typename TB_>
__global__ void __launch_bounds__(kT) k16_sub_norm(int64_t n16, const double* __restrict__ a, const TB_* __restrict__ bv,
                                                   double* __restrict__ outd, float* __restrict__ outf,
                                                   double* __restrict__ part) {
    __shared__ double red[(kT / 64) * KC];
    int64_t j0, j1;
    arn::block_range(n16, blockIdx.x, j0, j1);
    double acc[1] = {0.0};
    // 4 elements per thread and round, every load of a round issued before its use (one
    // load per element: one at a time left the kernel at 2.4 TB/s, r06n)
    constexpr int U = 4;
    for (int64_t e0 = j0 + threadIdx.x; e0 < j1; e0 += U * kT) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = e0 + (int64_t)u * kT;
            v[u] = e < j1 ? a[e] : 0.0;
        }
        if (bv)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t e = e0 + (int64_t)u * kT;
                if (e < j1) v[u] -= (double)bv[e];
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = e0 + (int64_t)u * kT;
            if (e >= j1) continue;
            double w = v[u];
            if (outd) outd[e] = w;
            if (outf) {
                const float f = (float)w;
                outf[e] = f;
                w = (double)f;
            }
            acc[0] = __builtin_fma(w, w, acc[0]);
        }
    }
    block_store16<1>(acc, 1, -1, red, part, blockIdx.x);
}

// per-column sums of a one-row partial set into out[c] (device or mapped host memory)
__global__ void __launch_bounds__(arn::kThreads) k16_rows(const double* __restrict__ part, double* __restrict__ out) {
    __shared__ double scratch[arn::kRedRows * 64];
    __shared__ double o[1];
    arn::reduce_rows(part + (size_t)blockIdx.x * kParts, kParts, kParts, 1, o, scratch);
    if (threadIdx.x == 0) out[blockIdx.x] = o[0];
}

// x[e] += sum_{k < used} y_c[k] V_k[e] (c = e % 16; y_c in column c's state block)
__global__ void __launch_bounds__(256) k16_axpy(int64_t n16, int used, const float* __restrict__ V, int64_t ldv,
                                                const double* __restrict__ st, int64_t sts, int m,
                                                double* __restrict__ x) {
    extern __shared__ double ys[];  // [k][c]
    const arn::Layout L(m);
    for (int f = threadIdx.x; f < used * KC; f += 256) ys[f] = st[(f % KC) * sts + L.y + f / KC];
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n16) return;
    const int c = (int)(e % KC);
    double a = x[e];
    for (int k = 0; k < used; ++k) a = __builtin_fma(ys[k * KC + c], (double)V[(size_t)k * ldv + e], a);
    x[e] = a;
}

// y += x (fp64); xf = (float)x (may be null)
__global__ void __launch_bounds__(256) k16_add(int64_t n, const double* __restrict__ x, double* __restrict__ y) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < n) y[e] += x[e];
}
__global__ void __launch_bounds__(256) k16_round(int64_t n, const double* __restrict__ x, float* __restrict__ y) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < n) y[e] = (float)x[e];
}

// rows (16 vectors of N, original order, stride ld) <-> N x 16 point-major tree order
__global__ void __launch_bounds__(256) k16_gather(int64_t N, const int* __restrict__ perm, const double* __restrict__ rows,
                                                  int64_t ld, double* __restrict__ pm) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N * KC) return;
    const int64_t k = e / KC;
    pm[e] = rows[(size_t)(e % KC) * ld + perm[k]];
}
__global__ void __launch_bounds__(256) k16_scatter(int64_t N, const int* __restrict__ perm, const double* __restrict__ pm,
                                                   double* __restrict__ rows, int64_t ld) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N * KC) return;
    const int64_t k = e / KC;
    rows[(size_t)(e % KC) * ld + perm[k]] = pm[e];
}

template <typename F>
inline void rows_dispatch(int nv, F&& f) {
    if (nv <= 8) f(std::integral_constant<int, 8>{});
    else if (nv <= 16) f(std::integral_constant<int, 16>{});
    else if (nv <= 24) f(std::integral_constant<int, 24>{});
    else if (nv <= 32) f(std::integral_constant<int, 32>{});
    else if (nv <= 40) f(std::integral_constant<int, 40>{});
    else f(std::integral_constant<int, kMaxRows>{});
}

}  // namespace arn16
}  // namespace aniso
