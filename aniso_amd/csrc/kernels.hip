// kernels.hip -- hand-written CDNA4 (gfx950) kernels for the device-side cache
// build of the anisotropic RTE integral operator (the apply kernels are in
// apply.hip).
//
// Reference behaviour (file:line under lowrank/aniso):
//   cache build  bbfmm.h:949-1039, KernelFactory.cpp:67-207, 240-267
// Both bbfmm instances (imag (e^-tau - 1) cos(m th)/r and real cos(m th)/r) share
// tree, lists, charges and translation operators, so one pass with the summed
// kernel e^-tau cos(m th)/r computes their sum (DESIGN.md "Merged kernels").
#include <hip/hip_runtime.h>

#include <cmath>

#include "device_common.hpp"

namespace aniso {

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

// imag_m + real_m (makeKernels, KernelFactory.cpp:240-267); a = source, b = target.
// m = kAttMode: the mode-independent factor e^-tau alone (0 at r = 0), the entry of
// the mode-shared cache.
__device__ double pair_kernel(const Params* __restrict__ P, const double* __restrict__ stcoef, int m, double ax,
                              double ay, double bx, double by) {
    double ddx = ax - bx, ddy = ay - by;
    double dist = sqrt(ddx * ddx + ddy * ddy);
    if (m == kAttMode) return dist == 0.0 ? 0.0 : exp(-line_integral(P, stcoef, ax, ay, bx, by));
    if (dist == 0.0) return m == 0 ? sigma_eval(P, stcoef, ax, ay) : 0.0;
    double gk = (m == 0) ? 1.0 / dist : cos(m * atan2(ddy, ddx)) / dist;
    double tau = line_integral(P, stcoef, ax, ay, bx, by);
    return exp(-tau) * gk;
}

__global__ void k_permute(int64_t N, const int* __restrict__ perm, const double* __restrict__ orig,
                          double* __restrict__ tree) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) tree[k] = orig[perm[k]];
}

// ----------------------------------------------------------------- cache build

// downPassCache's M2L blocks (bbfmm.h:959-975, 782-804) for all stored (target,
// source) pairs, K[t][s] = kernel(cheb_s(src), cheb_t(tgt)), column-major
// (pair*256 + s*16 + t), the layout k_m2l streams; pairTgt = ~target marks a
// canonical block (same layout, also read transposed).
__global__ void __launch_bounds__(256) k_cache_m2l(int64_t total, const int* __restrict__ pairTgt,
                                                   const int* __restrict__ src, const double* __restrict__ ncx,
                                                   const double* __restrict__ ncy, const double* __restrict__ nrx,
                                                   const double* __restrict__ nry, const double* __restrict__ stcoef,
                                                   const Params* __restrict__ P, int mode, double* __restrict__ K) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int64_t p = e >> 8;
    const int s = (int)((e >> 4) & 15), t = (int)(e & 15);
    int tn = pairTgt[p];
    const int sn = src[p];
    if (tn < 0) tn = ~tn;
    double bx = ncx[tn] + nrx[tn] * P->cheb[t & 3];
    double by = ncy[tn] + nry[tn] * P->cheb[t >> 2];
    double ax = ncx[sn] + nrx[sn] * P->cheb[s & 3];
    double ay = ncy[sn] + nry[sn] * P->cheb[s >> 2];
    K[e] = pair_kernel(P, stcoef, mode, ax, ay, bx, by);
}

// Mode-shared M2L cache: E[t][s] = e^-tau(cheb_s(src), cheb_t(tgt))
// for every directed (target, source) pair, column-major (pair*256 + s*16 + t), the
// layout k_m2l_hm streams (lane (column s, row quad) reads 32 contiguous bytes).
__global__ void __launch_bounds__(256) k_cache_att_m2l(int64_t total, const int* __restrict__ pairTgt,
                                                       const int* __restrict__ src, const double* __restrict__ ncx,
                                                       const double* __restrict__ ncy, const double* __restrict__ nrx,
                                                       const double* __restrict__ nry,
                                                       const double* __restrict__ stcoef,
                                                       const Params* __restrict__ P, double* __restrict__ E) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int64_t p = e >> 8;
    const int s = (int)((e >> 4) & 15), t = (int)(e & 15);
    const int tn = pairTgt[p], sn = src[p];
    double bx = ncx[tn] + nrx[tn] * P->cheb[t & 3];
    double by = ncy[tn] + nry[tn] * P->cheb[t >> 2];
    double ax = ncx[sn] + nrx[sn] * P->cheb[s & 3];
    double ay = ncy[sn] + nry[sn] * P->cheb[s >> 2];
    E[e] = pair_kernel(P, stcoef, kAttMode, ax, ay, bx, by);
}

// The mode-0 diagonal of the merged kernel, sigma_t at each point (evaluate(a),
// KernelFactory.cpp:260), tree order: the r = 0 entry the mode-shared near field
// adds apart from its blocks.
__global__ void k_sigma_diag(int64_t N, const double* __restrict__ pxT, const double* __restrict__ pyT,
                             const double* __restrict__ stcoef, const Params* __restrict__ P,
                             double* __restrict__ out) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) out[k] = sigma_eval(P, stcoef, pxT[k], pyT[k]);
}

// downPassCache's U/W blocks (bbfmm.h:991-1011): per target leaf, column-major
// nT4 x S (nT rounded up to a multiple of 4, zero rows) over the concatenated source points of its U then W members.
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
    const int nTs = (nT + 3) & ~3;  // rows padded to a multiple of 4 (32-B row quads in k_near)
    const int64_t total = (int64_t)nTs * S;
    for (int64_t e = threadIdx.x; e < total; e += blockDim.x) {
        int sc = (int)(e / nTs), t = (int)(e - (int64_t)sc * nTs);
        if (t >= nT) {
            Kl[e] = 0.0;
            continue;
        }
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

void launch_cache_m2l(int64_t npairs, const int* pairTgt, const int* src, const double* ncx, const double* ncy,
                      const double* nrx, const double* nry, const double* stcoef, const Params* P, int mode,
                      double* K, hipStream_t s) {
    if (npairs <= 0) return;
    int64_t total = npairs * 256;
    k_cache_m2l<<<blocks_for(total, 256), 256, 0, s>>>(total, pairTgt, src, ncx, ncy, nrx, nry, stcoef, P, mode, K);
    HIP_LAUNCH_CHECK();
}

void launch_cache_att_m2l(int64_t npairs, const int* pairTgt, const int* src, const double* ncx, const double* ncy,
                          const double* nrx, const double* nry, const double* stcoef, const Params* P, double* E,
                          hipStream_t s) {
    if (npairs <= 0) return;
    int64_t total = npairs * 256;
    k_cache_att_m2l<<<blocks_for(total, 256), 256, 0, s>>>(total, pairTgt, src, ncx, ncy, nrx, nry, stcoef, P, E);
    HIP_LAUNCH_CHECK();
}

void launch_sigma_diag(int64_t N, const double* pxT, const double* pyT, const double* stcoef, const Params* P,
                       double* out, hipStream_t s) {
    if (N <= 0) return;
    k_sigma_diag<<<blocks_for(N, 256), 256, 0, s>>>(N, pxT, pyT, stcoef, P, out);
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

// ---- halo exchange of the sharded apply (comm.hpp)
__global__ void k_halo_pack(int64_t n, int nb, const int64_t* __restrict__ pos, const int64_t* __restrict__ base,
                            const int64_t* __restrict__ stride, const double* __restrict__ x, int64_t ldx,
                            double* __restrict__ buf) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    for (int b = 0; b < nb; ++b) buf[base[j] + b * stride[j]] = x[(size_t)b * ldx + pos[j]];
}

__global__ void k_halo_unpack(int64_t n, int nb, const int64_t* __restrict__ pos, const int64_t* __restrict__ base,
                              const int64_t* __restrict__ stride, const double* __restrict__ buf,
                              double* __restrict__ x, int64_t ldx) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    for (int b = 0; b < nb; ++b) x[(size_t)b * ldx + pos[j]] = buf[base[j] + b * stride[j]];
}

void launch_halo_pack(int64_t n, int nb, const int64_t* pos, const int64_t* base, const int64_t* stride,
                      const double* x, int64_t ldx, double* buf, hipStream_t s) {
    if (n <= 0) return;
    k_halo_pack<<<blocks_for(n, 256), 256, 0, s>>>(n, nb, pos, base, stride, x, ldx, buf);
    HIP_LAUNCH_CHECK();
}

void launch_halo_unpack(int64_t n, int nb, const int64_t* pos, const int64_t* base, const int64_t* stride,
                        const double* buf, double* x, int64_t ldx, hipStream_t s) {
    if (n <= 0) return;
    k_halo_unpack<<<blocks_for(n, 256), 256, 0, s>>>(n, nb, pos, base, stride, buf, x, ldx);
    HIP_LAUNCH_CHECK();
}


}  // namespace aniso
