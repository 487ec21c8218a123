// corr_point.hpp -- the corrections of one target point (nearRemoval +
// refineAddOnFast + singularAddFast, KernelFactory.cpp:445-478, 662-709, 828-860):
// a 3x3-square stencil with translation-invariant d2 x 9 x d2 weights Wc (every mode
// term of the apply folded in on the host, Operator::corrTable) plus the singular term
// from the Legendre coefficients of the target's own square (O(d^4) moments, Wm).
// Shared by k_corr (neighbour charges from fT in HBM) and the near field's fused
// epilogue (k_near_hs: neighbour charges from its LDS source table); `charges(q9, c,
// f)` returns the K weighted charges of point c of neighbour square q9 = 3 (dr+1) +
// (dc+1), or false outside the grid; `cval(k, r)` the unweighted charge r of tree
// position k (cT, or the apply's input, k_near_hs).
#pragma once

#include "device_common.hpp"

namespace aniso {

template <int D, int K, class Charges, class CVal>
__device__ __forceinline__ void corr_point(int t, const Params* __restrict__ P, const int* __restrict__ iperm,
                                           CVal cval, const double* __restrict__ Wc,
                                           const double* __restrict__ Wm, int flags, Charges charges,
                                           double (&acc)[K]) {
    constexpr int D2 = D * D;
    const int sz = P->sz;
    const int sq = t / D2, tq = t - sq * D2;
    const int i = sq / sz, j = sq - i * sz;
#pragma unroll
    for (int r = 0; r < K; ++r) acc[r] = 0.0;
    if (flags & kStageStencil) {
#pragma unroll
        for (int dr = -1; dr <= 1; ++dr) {
            if (i + dr < 0 || i + dr >= sz) continue;
#pragma unroll
            for (int dc = -1; dc <= 1; ++dc) {
                if (j + dc < 0 || j + dc >= sz) continue;
                const int q9 = (dr + 1) * 3 + (dc + 1);
#pragma unroll
                for (int c = 0; c < D2; ++c) {
                    double f[K];
                    charges(q9, sq + dr * sz + dc, c, f);
                    const double* w = Wc + (((size_t)tq * 9 + q9) * D2 + c) * K * K;
#pragma unroll
                    for (int r = 0; r < K; ++r)
#pragma unroll
                        for (int bb = 0; bb < K; ++bb) acc[r] += w[r * K + bb] * f[bb];
                }
            }
        }
    }
    if (flags & kStageSing) {
        // shifted Legendre bases of the square (singularAddFast evaluates the
        // expansion at global coordinates, quirk 1): P_n(X + h u) = sum_a bx[n][a] u^a
        const double X = (0.5 + i) * P->dx, Y = (0.5 + j) * P->dx;
        double bx[D][D], by[D][D];
#pragma unroll
        for (int n = 0; n < D; ++n)
#pragma unroll
            for (int a = 0; a < D; ++a) {
                double sx = 0.0, sy = 0.0, px = 1.0, py = 1.0;
#pragma unroll
                for (int e2 = 0; e2 < D; ++e2) {
                    double cb = P->legB[(n * D + a) * D + e2];
                    sx += cb * px;
                    sy += cb * py;
                    px *= X;
                    py *= Y;
                }
                bx[n][a] = sx;
                by[n][a] = sy;
            }
        const int* itS = iperm + (size_t)sq * D2;  // the target square's points, tree positions
#pragma unroll 1
        for (int r = 0; r < K; ++r) {
            double hw[D2];
#pragma unroll
            for (int c = 0; c < D2; ++c) hw[c] = P->sqrtW[c] * cval((int64_t)itS[c], r);
            // Legendre coefficients cf_{n,k} = (interpolate * (sqrtW .* h))_{nk} / norm_nk,
            // contracted with the bases: pb[a][bb] = sum_{n >= a, k >= bb} cf_nk bx[n][a] by[k][bb]
            double pb[D][D];
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int bb = 0; bb < D; ++bb) pb[a][bb] = 0.0;
#pragma unroll
            for (int nk = 0; nk < D2; ++nk) {
                double c = 0.0;
#pragma unroll
                for (int q = 0; q < D2; ++q) c += P->interp[nk + q * D2] * hw[q];
                c *= P->coefScale[nk];
                const int n = nk / D, kk = nk % D;
#pragma unroll
                for (int a = 0; a < D; ++a)
#pragma unroll
                    for (int bb = 0; bb < D; ++bb)
                        if (a <= n && bb <= kk) pb[a][bb] += c * bx[n][a] * by[kk][bb];
            }
            const double* wm = Wm + ((size_t)tq * K * K + r) * D2;  // [tq][i][b = r][a][bb], i stride K D2
#pragma unroll
            for (int ii = 0; ii < K; ++ii) {
                double sg = 0.0;
#pragma unroll
                for (int ab = 0; ab < D2; ++ab) sg += pb[ab / D][ab % D] * wm[(size_t)ii * K * D2 + ab];
                acc[ii] += sg;
            }
        }
    }
}

}  // namespace aniso
