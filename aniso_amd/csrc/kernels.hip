// kernels.hip -- hand-written CDNA4 (gfx950) kernels for one apply of the
// anisotropic RTE integral operator and for its device-side cache build.
//
// Reference behaviour (file:line under lowrank/aniso):
//   apply        AnisoWrapper.cpp:92-136  (imag + real bbfmm, nearRemoval,
//                refineAddOnFast, singularAddFast, combine)
//   up pass      bbfmm.h:825-861          (P2M leaf transfer, M2M)
//   down pass    bbfmm.h:1041-1129        (M2L over V/X, L2L, U/W near, L2P)
//   cache build  bbfmm.h:949-1039, KernelFactory.cpp:67-207, 240-267
// Both bbfmm instances (imag (e^-tau - 1) cos(m th)/r and real cos(m th)/r) share
// tree, lists, charges and translation operators, so one pass with the summed
// kernel e^-tau cos(m th)/r computes their sum (DESIGN.md "Merged kernels").
#include <hip/hip_runtime.h>

#include <cmath>

#include "kernels.hpp"

namespace aniso {

#define HIP_LAUNCH_CHECK()                                                                  \
    do {                                                                                    \
        hipError_t e__ = hipGetLastError();                                                 \
        if (e__ != hipSuccess) throw_hip(e__, __FILE__, __LINE__);                          \
    } while (0)

[[noreturn]] void throw_hip(hipError_t e, const char* file, int line);

constexpr int kWave = 64;
typedef double dbl2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------- helpers

// std::tr1::legendre recurrence (libstdc++ __poly_legendre_p), values P_0..P_{d-1}
__device__ __forceinline__ void legendre_all(int d, double x, double* P) {
    P[0] = 1.0;
    if (d < 2) return;
    if (x == 1.0 || x == -1.0) {
        for (int l = 1; l < d; ++l) P[l] = (x == -1.0 && (l & 1)) ? -1.0 : 1.0;
        return;
    }
    P[1] = x;
    for (int l = 2; l < d; ++l) P[l] = 2.0 * x * P[l - 1] - P[l - 2] - (x * P[l - 1] - P[l - 2]) / (double)l;
}

// Chebyshev interpolant S(s, c_i) = (-1 + 2 sum_l T_l(s) T_l(c_i)) / np  (bbfmm.h:635-656, 737-748)
__device__ __forceinline__ void cheb_weights(const Params* __restrict__ P, double s, double* S) {
    double T[kNP];
    T[0] = 1.0;
    T[1] = s;
#pragma unroll
    for (int l = 2; l < kNP; ++l) T[l] = 2.0 * s * T[l - 1] - T[l - 2];
#pragma unroll
    for (int i = 0; i < kNP; ++i) {
        double acc = 0.0;
#pragma unroll
        for (int l = 0; l < kNP; ++l) acc += T[l] * P->tnode[i + l * kNP];
        S[i] = (2.0 * acc - 1.0) * (1.0 / kNP);
    }
}

// integral_helper (KernelFactory.cpp:174-190): d-point Gauss rule on one piece
// lying in one square; sigma_t's Legendre expansion is evaluated at GLOBAL
// coordinates (reference quirk).  stcoef already carries 1/legendreNorms.
__device__ double sigma_piece(const Params* __restrict__ P, const double* __restrict__ stcoef, double xa, double ya,
                              double xb, double yb) {
    const int sz = P->sz, d = P->d, d2 = P->d2;
    double mx = (xa + xb) / 2, my = (ya + yb) / 2;
    int col = (int)floor(mx * sz), row = (int)floor(my * sz);
    col = col < 0 ? 0 : (col >= sz ? sz - 1 : col);
    row = row < 0 ? 0 : (row >= sz ? sz - 1 : row);
    const double* c = stcoef + (size_t)(col * sz + row) * d2;
    double ret = 0.0;
    double Px[kMaxD], Py[kMaxD];
    for (int i = 0; i < d; ++i) {
        double x = mx + (xa - xb) / 2 * P->gx[i];
        double y = my + (ya - yb) / 2 * P->gx[i];
        legendre_all(d, x, Px);
        legendre_all(d, y, Py);
        double dot = 0.0;
        for (int n = 0; n < d; ++n) {
            double rowdot = 0.0;
            for (int k = 0; k < d; ++k) rowdot += Py[k] * c[n * d + k];
            dot += Px[n] * rowdot;
        }
        ret += dot * P->gw[i];
    }
    double ddx = xa - xb, ddy = ya - yb;
    return ret * sqrt(ddx * ddx + ddy * ddy) / 2.0;
}

// lineIntegral (KernelFactory.cpp:67-166).  The reference splits the segment at
// midpoints and grid lines and applies the Gauss rule per piece; the integrand is
// a polynomial of degree <= 2d-2 inside every square, so the d-point rule is exact
// on any piece inside one square and the value is independent of where the pieces
// are cut.  We walk the grid cells the segment crosses (DDA) instead: same
// integral, no recursion, bounded loop (one iteration per crossed square).
__device__ double line_integral(const Params* __restrict__ P, const double* __restrict__ stcoef, double x0,
                                double y0, double x1, double y1) {
    const int sz = P->sz;
    const double dx = P->dx;
    int c0 = (int)floor(x0 * sz), r0 = (int)floor(y0 * sz);
    int c1 = (int)floor(x1 * sz), r1 = (int)floor(y1 * sz);
    if (c0 == c1 && r0 == r1) return sigma_piece(P, stcoef, x0, y0, x1, y1);
    const double ddx = x1 - x0, ddy = y1 - y0;
    const double INF = 1e300;
    double tmx = INF, tdx = INF, tmy = INF, tdy = INF;
    if (ddx != 0.0) {
        double xb = (ddx > 0 ? (c0 + 1) : c0) * dx;
        tmx = (xb - x0) / ddx;
        tdx = dx / fabs(ddx);
    }
    if (ddy != 0.0) {
        double yb = (ddy > 0 ? (r0 + 1) : r0) * dx;
        tmy = (yb - y0) / ddy;
        tdy = dx / fabs(ddy);
    }
    double t0 = 0.0, sum = 0.0, xa = x0, ya = y0;
    const int guard = abs(c1 - c0) + abs(r1 - r0) + 4;
    for (int it = 0; it < guard; ++it) {
        double tn = fmin(fmin(tmx, tmy), 1.0);
        bool last = tn >= 1.0;
        double xb = last ? x1 : x0 + tn * ddx;
        double yb = last ? y1 : y0 + tn * ddy;
        if (tn > t0) sum += sigma_piece(P, stcoef, xa, ya, xb, yb);
        if (last) return sum;
        if (tmx <= tn) tmx += tdx;
        if (tmy <= tn) tmy += tdy;
        t0 = tn;
        xa = xb;
        ya = yb;
    }
    return sum + sigma_piece(P, stcoef, xa, ya, x1, y1);
}

// evaluate (KernelFactory.cpp:193-207): sigma_t at a point, global-coordinate Legendre
__device__ double sigma_eval(const Params* __restrict__ P, const double* __restrict__ stcoef, double x, double y) {
    const int sz = P->sz, d = P->d;
    int col = (int)floor(x * sz), row = (int)floor(y * sz);
    col = col < 0 ? 0 : (col >= sz ? sz - 1 : col);
    row = row < 0 ? 0 : (row >= sz ? sz - 1 : row);
    const double* c = stcoef + (size_t)(col * sz + row) * P->d2;
    double Px[kMaxD], Py[kMaxD];
    legendre_all(d, x, Px);
    legendre_all(d, y, Py);
    double s = 0.0;
    for (int n = 0; n < d; ++n)
        for (int k = 0; k < d; ++k) s += Px[n] * Py[k] * c[n * d + k];
    return s;
}

// imag_m + real_m (makeKernels, KernelFactory.cpp:240-267); a = source, b = target
__device__ double pair_kernel(const Params* __restrict__ P, const double* __restrict__ stcoef, int m, double ax,
                              double ay, double bx, double by) {
    double ddx = ax - bx, ddy = ay - by;
    double dist = sqrt(ddx * ddx + ddy * ddy);
    if (dist == 0.0) return m == 0 ? sigma_eval(P, stcoef, ax, ay) : 0.0;
    double gk = (m == 0) ? 1.0 / dist : cos(m * atan2(ddy, ddx)) / dist;
    double tau = line_integral(P, stcoef, ax, ay, bx, by);
    return exp(-tau) * gk;
}

// ----------------------------------------------------------------- apply kernels

__global__ void k_prepare(int64_t N, const int* __restrict__ perm, const double* __restrict__ charge,
                          const double* __restrict__ w, double* __restrict__ fT, double* __restrict__ fO) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    int t = perm[k];
    fT[k] = charge[t] * w[t];
    fO[k] = charge[k] * w[k];
}

// P2M: nodeCharge = R^T q, R(k, j*np+i) = Sx(k,i) Sy(k,j)  (bbfmm.h:832-844)
__global__ void k_p2m(int nl, const int* __restrict__ leaves, const int64_t* __restrict__ begin,
                      const int64_t* __restrict__ count, const double* __restrict__ ncx,
                      const double* __restrict__ ncy, const double* __restrict__ nrx, const double* __restrict__ nry,
                      const double* __restrict__ pxT, const double* __restrict__ pyT, const double* __restrict__ fT,
                      const Params* __restrict__ P, double* __restrict__ mult) {
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    int li = gid >> 4, p = gid & 15;
    if (li >= nl) return;
    int n = leaves[li];
    int i = p & 3, j = p >> 2;
    double cx = ncx[n], cy = ncy[n], rx = nrx[n], ry = nry[n];
    int64_t b = begin[n], e = b + count[n];
    double acc = 0.0;
    for (int64_t k = b; k < e; ++k) {
        double Sx[kNP], Sy[kNP];
        cheb_weights(P, (pxT[k] - cx) / rx, Sx);
        cheb_weights(P, (pyT[k] - cy) / ry, Sy);
        acc += Sx[i] * Sy[j] * fT[k];
    }
    mult[(size_t)n * kRank + p] = acc;
}

// M2M: parent += R[slot]^T child for non-empty children  (bbfmm.h:855-859)
__global__ void k_m2m(int nn, const int* __restrict__ nodes, const int4* __restrict__ child,
                      const int64_t* __restrict__ count, const Params* __restrict__ P, double* __restrict__ mult) {
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    int ni = gid >> 4, c = gid & 15;
    if (ni >= nn) return;
    int n = nodes[ni];
    int4 ch = child[n];
    int cs[4] = {ch.x, ch.y, ch.z, ch.w};
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (count[cs[i]] == 0) continue;
        const double* cm = mult + (size_t)cs[i] * kRank;
        const double* R = P->R[i] + (size_t)c * kRank;
#pragma unroll
        for (int r = 0; r < kRank; ++r) acc += R[r] * cm[r];
    }
    mult[(size_t)n * kRank + c] = acc;
}

// M2L over the V then X lists with the cached merged 16x16 operators
// (bbfmm.h:1051-1065).  HBM-bound stream: one wave per target node, each pair's
// 2 KB operator is read as 64 lanes x 32 contiguous bytes (two dwordx4 loads).
// Lane l owns row t = l>>2 and columns 4(l&3)..4(l&3)+3.
__global__ void __launch_bounds__(256) k_m2l(int ntgt, const int* __restrict__ tgt, const int64_t* __restrict__ ptr,
                                             const int* __restrict__ src, const double* __restrict__ K,
                                             const double* __restrict__ mult, double* __restrict__ local) {
    int wave = (blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    int lane = threadIdx.x & (kWave - 1);
    if (wave >= ntgt) return;
    int n = tgt[wave];
    int t = lane >> 2, q = lane & 3;
    int64_t p0 = ptr[wave], p1 = ptr[wave + 1];
    double acc0 = 0.0, acc1 = 0.0;
    int64_t p = p0;
    for (; p + 1 < p1; p += 2) {
        const dbl2* ka = reinterpret_cast<const dbl2*>(K + (size_t)p * 256 + t * 16 + q * 4);
        const dbl2* kb = reinterpret_cast<const dbl2*>(K + (size_t)(p + 1) * 256 + t * 16 + q * 4);
        dbl2 a0 = __builtin_nontemporal_load(ka), a1 = __builtin_nontemporal_load(ka + 1);
        dbl2 b0 = __builtin_nontemporal_load(kb), b1 = __builtin_nontemporal_load(kb + 1);
        const double2* ma = reinterpret_cast<const double2*>(mult + (size_t)src[p] * kRank + q * 4);
        const double2* mb = reinterpret_cast<const double2*>(mult + (size_t)src[p + 1] * kRank + q * 4);
        double2 ma0 = ma[0], ma1 = ma[1], mb0 = mb[0], mb1 = mb[1];
        acc0 += a0.x * ma0.x + a0.y * ma0.y + a1.x * ma1.x + a1.y * ma1.y;
        acc1 += b0.x * mb0.x + b0.y * mb0.y + b1.x * mb1.x + b1.y * mb1.y;
    }
    if (p < p1) {
        const dbl2* ka = reinterpret_cast<const dbl2*>(K + (size_t)p * 256 + t * 16 + q * 4);
        dbl2 a0 = __builtin_nontemporal_load(ka), a1 = __builtin_nontemporal_load(ka + 1);
        const double2* ma = reinterpret_cast<const double2*>(mult + (size_t)src[p] * kRank + q * 4);
        double2 ma0 = ma[0], ma1 = ma[1];
        acc0 += a0.x * ma0.x + a0.y * ma0.y + a1.x * ma1.x + a1.y * ma1.y;
    }
    double acc = acc0 + acc1;
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (q == 0) local[(size_t)n * kRank + t] = acc;
}

// L2L: local += R[slot] * parent.local  (bbfmm.h:1070-1071)
__global__ void k_l2l(int nn, const int* __restrict__ nodes, const int* __restrict__ parent,
                      const int* __restrict__ slot, const Params* __restrict__ P, double* __restrict__ local) {
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    int ni = gid >> 4, r = gid & 15;
    if (ni >= nn) return;
    int n = nodes[ni];
    const double* pl = local + (size_t)parent[n] * kRank;
    const double* R = P->R[slot[n]];
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < kRank; ++c) acc += R[r + c * kRank] * pl[c];
    local[(size_t)n * kRank + r] += acc;
}

// U/W near field + L2P for one target leaf per wave (bbfmm.h:1081-1113).  The
// leaf's cached block is column-major nT x S (S = all U/W source points), read
// as consecutive columns: lanes (t, column phase), t on the low lane bits.
__global__ void __launch_bounds__(256) k_near_l2p(
    int nl, const int* __restrict__ leaves, const int64_t* __restrict__ nearPtr, const int* __restrict__ nearSrc,
    const int64_t* __restrict__ nearKOff, const double* __restrict__ K, const int64_t* __restrict__ begin,
    const int64_t* __restrict__ count, const double* __restrict__ ncx, const double* __restrict__ ncy,
    const double* __restrict__ nrx, const double* __restrict__ nry, const double* __restrict__ pxT,
    const double* __restrict__ pyT, const double* __restrict__ fT, const double* __restrict__ local,
    const int* __restrict__ perm, const Params* __restrict__ P, int maxS, int flags, double* __restrict__ out) {
    extern __shared__ double sh[];
    const int wv = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    const int li = blockIdx.x * (blockDim.x / kWave) + wv;
    const bool active = li < nl;
    double* fs = sh + (size_t)wv * maxS;
    int n = 0, nT = 0, S = 0;
    int64_t tb = 0;
    if (active) {
        n = leaves[li];
        nT = (int)count[n];
        tb = begin[n];
        // stage the source charges of all U/W members (each a contiguous tree range)
        for (int64_t j = nearPtr[li]; j < nearPtr[li + 1]; ++j) {
            int s = nearSrc[j];
            int64_t sb = begin[s];
            int sc = (int)count[s];
            for (int k = lane; k < sc; k += kWave) fs[S + k] = fT[sb + k];
            S += sc;
        }
    }
    __syncthreads();
    if (!active) return;
    const double* Kl = K + nearKOff[li];
    const int nTp = nT <= 16 ? 16 : (nT <= 32 ? 32 : 64);
    const int cps = kWave / nTp;
    const int sph = lane / nTp;
    for (int tc = 0; tc < nT; tc += kWave) {
        const int t = tc + (lane & (nTp - 1));
        double acc = 0.0;
        if ((flags & kStageNear) && t < nT) {
            int s = sph;
            for (; s + cps < S; s += 2 * cps) {
                double k0 = __builtin_nontemporal_load(Kl + (size_t)s * nT + t);
                double k1 = __builtin_nontemporal_load(Kl + (size_t)(s + cps) * nT + t);
                acc += k0 * fs[s] + k1 * fs[s + cps];
            }
            if (s < S) acc += __builtin_nontemporal_load(Kl + (size_t)s * nT + t) * fs[s];
        }
        for (int off = nTp; off < kWave; off <<= 1) acc += __shfl_xor(acc, off);
        if (sph == 0 && t < nT) {
            if (flags & kStageFar) {
                double Sx[kNP], Sy[kNP];
                cheb_weights(P, (pxT[tb + t] - ncx[n]) / nrx[n], Sx);
                cheb_weights(P, (pyT[tb + t] - ncy[n]) / nry[n], Sy);
                const double* L = local + (size_t)n * kRank;
                double l2p = 0.0;
#pragma unroll
                for (int j = 0; j < kNP; ++j)
#pragma unroll
                    for (int i = 0; i < kNP; ++i) l2p += Sx[i] * Sy[j] * L[j * kNP + i];
                acc += l2p;
            }
            out[perm[tb + t]] = acc;
        }
    }
}

// Corrections (nearRemoval + refineAddOnFast + singularAddFast,
// KernelFactory.cpp:445-478, 662-709, 828-860) as a 3x3-square stencil with
// per-mode translation-invariant d2 x 9 x d2 weights, plus the singular term
// from Legendre coefficients of the target's own square (O(d^4) moments), then
// the final 1/(2 pi) scale (AnisoWrapper.cpp:129-130).
template <int D>
__global__ void __launch_bounds__(256) k_corr(int64_t b, int64_t e, const int* __restrict__ perm,
                                              const double* __restrict__ charge, const double* __restrict__ fO,
                                              const double* __restrict__ C, const double* __restrict__ mu,
                                              const Params* __restrict__ P, int flags, double scale,
                                              double* __restrict__ out) {
    constexpr int D2 = D * D;
    int64_t k = b + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= e) return;
    const int t = perm[k];
    const int sz = P->sz;
    const int sq = t / D2, tq = t - sq * D2;
    const int i = sq / sz, j = sq - i * sz;
    double acc = 0.0;
    if (flags & kStageStencil) {
#pragma unroll
        for (int dr = -1; dr <= 1; ++dr) {
            if (i + dr < 0 || i + dr >= sz) continue;
#pragma unroll
            for (int dc = -1; dc <= 1; ++dc) {
                if (j + dc < 0 || j + dc >= sz) continue;
                const int q9 = (dr + 1) * 3 + (dc + 1);
                const double* w = C + ((size_t)tq * 9 + q9) * D2;
                const double* f = fO + (size_t)(sq + dr * sz + dc) * D2;
#pragma unroll
                for (int c = 0; c < D2; ++c) acc += w[c] * f[c];
            }
        }
    }
    if (flags & kStageSing) {
        const double* h = charge + (size_t)sq * D2;
        double hw[D2];
#pragma unroll
        for (int c = 0; c < D2; ++c) hw[c] = P->sqrtW[c] * h[c];
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
        const double* m = mu + (size_t)tq * D * D;
        double sing = 0.0;
#pragma unroll
        for (int n = 0; n < D; ++n)
#pragma unroll
            for (int kk = 0; kk < D; ++kk) {
                // Legendre coefficient c_{n,k} = (interpolate * (sqrtW .* h))_{nk} / norm_nk
                double c = 0.0;
#pragma unroll
                for (int q = 0; q < D2; ++q) c += P->interp[(n * D + kk) + q * D2] * hw[q];
                c *= P->coefScale[n * D + kk];
                double mom = 0.0;
#pragma unroll
                for (int a = 0; a <= n; ++a)
#pragma unroll
                    for (int bb = 0; bb <= kk; ++bb) mom += bx[n][a] * by[kk][bb] * m[a * D + bb];
                sing += c * mom;
            }
        acc += sing;
    }
    out[t] = (out[t] + acc) * scale;
}

__global__ void k_permute(int64_t N, const int* __restrict__ perm, const double* __restrict__ orig,
                          double* __restrict__ tree) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) tree[k] = orig[perm[k]];
}

// ----------------------------------------------------------------- cache build

// downPassCache's M2L blocks (bbfmm.h:959-975, 782-804) for all (target, source)
// pairs: entry e = pair*256 + t*16 + s, K[t][s] = kernel(cheb_s(src), cheb_t(tgt)).
__global__ void __launch_bounds__(256) k_cache_m2l(int64_t total, const int* __restrict__ pairTgt,
                                                   const int* __restrict__ src, const double* __restrict__ ncx,
                                                   const double* __restrict__ ncy, const double* __restrict__ nrx,
                                                   const double* __restrict__ nry, const double* __restrict__ stcoef,
                                                   const Params* __restrict__ P, int mode, double* __restrict__ K) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int64_t p = e >> 8;
    int t = (int)((e >> 4) & 15), s = (int)(e & 15);
    int tn = pairTgt[p], sn = src[p];
    double bx = ncx[tn] + nrx[tn] * P->cheb[t & 3];
    double by = ncy[tn] + nry[tn] * P->cheb[t >> 2];
    double ax = ncx[sn] + nrx[sn] * P->cheb[s & 3];
    double ay = ncy[sn] + nry[sn] * P->cheb[s >> 2];
    K[e] = pair_kernel(P, stcoef, mode, ax, ay, bx, by);
}

// downPassCache's U/W blocks (bbfmm.h:991-1011): per target leaf, column-major
// nT x S over the concatenated source points of its U then W members.
__global__ void __launch_bounds__(256) k_cache_near(int nl, const int* __restrict__ leaves,
                                                    const int64_t* __restrict__ nearPtr,
                                                    const int* __restrict__ nearSrc,
                                                    const int64_t* __restrict__ nearKOff,
                                                    const int64_t* __restrict__ begin,
                                                    const int64_t* __restrict__ count, const double* __restrict__ pxT,
                                                    const double* __restrict__ pyT, const double* __restrict__ stcoef,
                                                    const Params* __restrict__ P, int mode, int maxSrc,
                                                    double* __restrict__ K) {
    extern __shared__ int64_t shi[];
    int64_t* sBeg = shi;
    int* sOff = reinterpret_cast<int*>(shi + maxSrc);
    const int li = blockIdx.x;
    if (li >= nl) return;
    const int n = leaves[li];
    const int nT = (int)count[n];
    const int64_t tb = begin[n];
    const int64_t j0 = nearPtr[li];
    const int ns = (int)(nearPtr[li + 1] - j0);
    if (threadIdx.x == 0) {
        int off = 0;
        for (int j = 0; j < ns; ++j) {
            int s = nearSrc[j0 + j];
            sBeg[j] = begin[s];
            sOff[j] = off;
            off += (int)count[s];
        }
        sOff[ns] = off;
    }
    __syncthreads();
    const int S = sOff[ns];
    double* Kl = K + nearKOff[li];
    const int64_t total = (int64_t)nT * S;
    for (int64_t e = threadIdx.x; e < total; e += blockDim.x) {
        int sc = (int)(e / nT), t = (int)(e - (int64_t)sc * nT);
        int j = 0;
        while (sOff[j + 1] <= sc) ++j;
        int64_t sp = sBeg[j] + (sc - sOff[j]);
        int64_t tp = tb + t;
        Kl[e] = pair_kernel(P, stcoef, mode, pxT[sp], pyT[sp], pxT[tp], pyT[tp]);
    }
}

__global__ void k_line_integrals(int n, const double* __restrict__ seg, const double* __restrict__ stcoef,
                                 const Params* __restrict__ P, double* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = line_integral(P, stcoef, seg[4 * i], seg[4 * i + 1], seg[4 * i + 2], seg[4 * i + 3]);
}

// ----------------------------------------------------------------- launchers

static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

void launch_prepare(int64_t N, const int* perm, const double* charge, const double* w, double* fT, double* fO,
                    hipStream_t s) {
    if (N <= 0) return;
    k_prepare<<<blocks_for(N, 256), 256, 0, s>>>(N, perm, charge, w, fT, fO);
    HIP_LAUNCH_CHECK();
}

void launch_p2m(int nl, const int* leaves, const int64_t* begin, const int64_t* count, const double* ncx,
                const double* ncy, const double* nrx, const double* nry, const double* pxT, const double* pyT,
                const double* fT, const Params* P, double* mult, hipStream_t s) {
    if (nl <= 0) return;
    k_p2m<<<blocks_for((int64_t)nl * 16, 256), 256, 0, s>>>(nl, leaves, begin, count, ncx, ncy, nrx, nry, pxT, pyT,
                                                            fT, P, mult);
    HIP_LAUNCH_CHECK();
}

void launch_m2m(int n, const int* nodes, const int4* child, const int64_t* count, const Params* P, double* mult,
                hipStream_t s) {
    if (n <= 0) return;
    k_m2m<<<blocks_for((int64_t)n * 16, 256), 256, 0, s>>>(n, nodes, child, count, P, mult);
    HIP_LAUNCH_CHECK();
}

void launch_m2l(int ntgt, const int* tgt, const int64_t* ptr, const int* src, const double* K, const double* mult,
                double* local, hipStream_t s) {
    if (ntgt <= 0) return;
    k_m2l<<<blocks_for((int64_t)ntgt * kWave, 256), 256, 0, s>>>(ntgt, tgt, ptr, src, K, mult, local);
    HIP_LAUNCH_CHECK();
}

void launch_l2l(int n, const int* nodes, const int* parent, const int* slot, const Params* P, double* local,
                hipStream_t s) {
    if (n <= 0) return;
    k_l2l<<<blocks_for((int64_t)n * 16, 256), 256, 0, s>>>(n, nodes, parent, slot, P, local);
    HIP_LAUNCH_CHECK();
}

void launch_near_l2p(int nl, const int* leaves, const int64_t* nearPtr, const int* nearSrc, const int64_t* nearKOff,
                     const double* K, const int64_t* begin, const int64_t* count, const double* ncx,
                     const double* ncy, const double* nrx, const double* nry, const double* pxT, const double* pyT,
                     const double* fT, const double* local, const int* perm, const Params* P, int maxS, int flags,
                     double* out, hipStream_t s) {
    if (nl <= 0) return;
    int wpb = maxS * 8 * 4 <= 48 * 1024 ? 4 : 1;
    size_t shm = (size_t)wpb * (maxS > 0 ? maxS : 1) * sizeof(double);
    k_near_l2p<<<blocks_for(nl, wpb), wpb * kWave, shm, s>>>(nl, leaves, nearPtr, nearSrc, nearKOff, K, begin, count,
                                                            ncx, ncy, nrx, nry, pxT, pyT, fT, local, perm, P,
                                                            maxS > 0 ? maxS : 1, flags, out);
    HIP_LAUNCH_CHECK();
}

void launch_corr(int d, int64_t b, int64_t e, const int* perm, const double* charge, const double* fO, const double* C,
                 const double* mu, const Params* P, int flags, double scale, double* out, hipStream_t s) {
    if (e <= b) return;
    unsigned nb = blocks_for(e - b, 256);
    switch (d) {
        case 1: k_corr<1><<<nb, 256, 0, s>>>(b, e, perm, charge, fO, C, mu, P, flags, scale, out); break;
        case 2: k_corr<2><<<nb, 256, 0, s>>>(b, e, perm, charge, fO, C, mu, P, flags, scale, out); break;
        case 3: k_corr<3><<<nb, 256, 0, s>>>(b, e, perm, charge, fO, C, mu, P, flags, scale, out); break;
        case 4: k_corr<4><<<nb, 256, 0, s>>>(b, e, perm, charge, fO, C, mu, P, flags, scale, out); break;
        case 5: k_corr<5><<<nb, 256, 0, s>>>(b, e, perm, charge, fO, C, mu, P, flags, scale, out); break;
        case 6: k_corr<6><<<nb, 256, 0, s>>>(b, e, perm, charge, fO, C, mu, P, flags, scale, out); break;
        default: throw_hip(hipErrorInvalidValue, __FILE__, __LINE__);
    }
    HIP_LAUNCH_CHECK();
}

void launch_cache_m2l(int64_t npairs, const int* pairTgt, const int* src, const double* ncx, const double* ncy,
                      const double* nrx, const double* nry, const double* stcoef, const Params* P, int mode,
                      double* K, hipStream_t s) {
    if (npairs <= 0) return;
    int64_t total = npairs * 256;
    k_cache_m2l<<<blocks_for(total, 256), 256, 0, s>>>(total, pairTgt, src, ncx, ncy, nrx, nry, stcoef, P, mode, K);
    HIP_LAUNCH_CHECK();
}

void launch_cache_near(int nl, const int* leaves, const int64_t* nearPtr, const int* nearSrc, const int64_t* nearKOff,
                       const int64_t* begin, const int64_t* count, const double* pxT, const double* pyT,
                       const double* stcoef, const Params* P, int mode, int maxSrc, double* K, hipStream_t s) {
    if (nl <= 0) return;
    size_t shm = (size_t)maxSrc * sizeof(int64_t) + (size_t)(maxSrc + 1) * sizeof(int);
    k_cache_near<<<nl, 256, shm, s>>>(nl, leaves, nearPtr, nearSrc, nearKOff, begin, count, pxT, pyT, stcoef, P, mode,
                                      maxSrc, K);
    HIP_LAUNCH_CHECK();
}

void launch_permute(int64_t N, const int* perm, const double* orig, double* tree, hipStream_t s) {
    if (N <= 0) return;
    k_permute<<<blocks_for(N, 256), 256, 0, s>>>(N, perm, orig, tree);
    HIP_LAUNCH_CHECK();
}

void launch_line_integrals(int n, const double* seg, const double* stcoef, const Params* P, double* out,
                           hipStream_t s) {
    if (n <= 0) return;
    k_line_integrals<<<blocks_for(n, 256), 256, 0, s>>>(n, seg, stcoef, P, out);
    HIP_LAUNCH_CHECK();
}

}  // namespace aniso
