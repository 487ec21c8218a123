// mrhs_corr.hpp -- the per-point corrections of the 16-right-hand-side MFMA
// operators (f32op.hip, f64op.hip).
#pragma once

#include "device_common.hpp"

namespace aniso {

// The corrections of one apply (nearRemoval + refineAddOn + singularAdd,
// KernelFactory.cpp:445-478, 662-709, 828-860) for 16 right-hand sides: the mode's
// stencil C (d2 x 9 x d2) and singular moments mu (d2 x d x d) as k_corr (apply.hip),
// one thread per point (its 16 right-hand sides as one 16-T row), fp64 arithmetic
// on the T charges; Y -= scale corr.  T = float (config 5's inner operator,
// f32op.hip) or double (the fp64 MFMA operator, f64op.hip).
template <typename T, int D>
__global__ void __launch_bounds__(256) k16_corr(int64_t N, const int* __restrict__ perm, const int* __restrict__ iperm,
                                                const T* __restrict__ cT, const T* __restrict__ fT,
                                                const double* __restrict__ C, const double* __restrict__ mu,
                                                const Params* __restrict__ P, int flags, T scale,
                                                T* __restrict__ Y) {
    constexpr int D2 = D * D;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    const int t = perm[k];
    const int sz = P->sz;
    const int sq = t / D2, tq = t - sq * D2;
    const int i = sq / sz, jj = sq - i * sz;
    double acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0;
    if (flags & kStageStencil) {
        for (int dr = -1; dr <= 1; ++dr) {
            if (i + dr < 0 || i + dr >= sz) continue;
            for (int dc = -1; dc <= 1; ++dc) {
                if (jj + dc < 0 || jj + dc >= sz) continue;
                const int q9 = (dr + 1) * 3 + (dc + 1);
                const int* it = iperm + (size_t)(sq + dr * sz + dc) * D2;
#pragma unroll
                for (int c = 0; c < D2; ++c) {
                    const double w = C[((size_t)tq * 9 + q9) * D2 + c];
                    const T* f = fT + (size_t)it[c] * 16;
#pragma unroll
                    for (int j = 0; j < 16; ++j) acc[j] += w * (double)f[j];
                }
            }
        }
    }
    if (flags & kStageSing) {
        const double Xc = (0.5 + i) * P->dx, Yc = (0.5 + jj) * P->dx;
        double bx[D][D], by[D][D];
#pragma unroll
        for (int nn = 0; nn < D; ++nn)
#pragma unroll
            for (int a = 0; a < D; ++a) {
                double sx = 0.0, sy = 0.0, px = 1.0, py = 1.0;
#pragma unroll
                for (int e2 = 0; e2 < D; ++e2) {
                    const double cb = P->legB[(nn * D + a) * D + e2];
                    sx += cb * px;
                    sy += cb * py;
                    px *= Xc;
                    py *= Yc;
                }
                bx[nn][a] = sx;
                by[nn][a] = sy;
            }
        // g[q] = sum_ab (basis products of coefficient nk) . mu: the singular term is
        // linear in the square's charges, sing_j = sum_q g[q] cT[q][j]
        double g[D2];
#pragma unroll
        for (int q = 0; q < D2; ++q) g[q] = 0.0;
#pragma unroll
        for (int nk = 0; nk < D2; ++nk) {
            const int nn = nk / D, kk = nk % D;
            double m = 0.0;  // sum over a <= nn, bb <= kk of bx by mu
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int bb = 0; bb < D; ++bb)
                    if (a <= nn && bb <= kk) m += bx[nn][a] * by[kk][bb] * mu[(size_t)tq * D2 + a * D + bb];
            m *= P->coefScale[nk];
#pragma unroll
            for (int q = 0; q < D2; ++q) g[q] += m * P->interp[nk + q * D2] * P->sqrtW[q];
        }
        const int* itS = iperm + (size_t)sq * D2;
#pragma unroll
        for (int q = 0; q < D2; ++q) {
            const T* c16 = cT + (size_t)itS[q] * 16;
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] += g[q] * (double)c16[j];
        }
    }
    T* y = Y + (size_t)k * 16;
#pragma unroll
    for (int j = 0; j < 16; ++j) y[j] -= scale * (T)acc[j];
}

}  // namespace aniso
