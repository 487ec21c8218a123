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

#include "host.hpp"  // kMaxCanon
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

// One Chebyshev interpolant weight S(s, c_i) (same arithmetic as cheb_weights).
__device__ __forceinline__ double cheb_weight1(const Params* __restrict__ P, double s, int i) {
    double T[kNP];
    T[0] = 1.0;
    T[1] = s;
#pragma unroll
    for (int l = 2; l < kNP; ++l) T[l] = 2.0 * s * T[l - 1] - T[l - 2];
    double acc = 0.0;
#pragma unroll
    for (int l = 0; l < kNP; ++l) acc += T[l] * P->tnode[i + l * kNP];
    return (2.0 * acc - 1.0) * (1.0 / kNP);
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

#ifdef ANISO_PROBE  // development build only (make probe): phase stamps of workgroup 0..kProbeWG-1
constexpr int kProbeWG = 2048;
__device__ unsigned long long g_probe[2][kProbeWG][8];
#define ANISO_STAMP(K, W, I)                                                     \
    do {                                                                          \
        if (threadIdx.x == 0 && (W) < kProbeWG) g_probe[K][W][I] = wall_clock64(); \
    } while (0)
extern "C" int aniso_probe_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_probe), sizeof(g_probe));
}
#else
#define ANISO_STAMP(K, W, I) \
    do {                  \
    } while (0)
#endif

// Output slot of tree position k: the original index perm[k] (original-order
// output) or the owned tree-order slice k - obase (operm == nullptr).
__device__ __forceinline__ int64_t out_index(const int* __restrict__ operm, int64_t obase, int64_t k) {
    return operm ? (int64_t)operm[k] : k - obase;
}

// Weighted charges in tree order: c = x_tree[k] (treeIn) or charge[perm[k]], times
// sigma_s in tree order when given; fT[k] = c w_T[k] (FMM and stencil charges),
// cT[k] = c (singular term).  The up pass does this inside its P2M; this kernel
// covers a tree without up-pass tiers (a lone leaf).
__device__ __forceinline__ double input_charge(const double* __restrict__ xin, int treeIn, const int* __restrict__ perm,
                                               const double* __restrict__ sigT, int64_t k) {
    const double c = treeIn ? xin[k] : xin[perm[k]];
    return sigT ? c * sigT[k] : c;
}

__global__ void k_prepare(int64_t N, const double* __restrict__ xin, int treeIn, const int* __restrict__ perm,
                          const double* __restrict__ sigT, const double* __restrict__ wT, double* __restrict__ fT,
                          double* __restrict__ cT) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    const double c = input_charge(xin, treeIn, perm, sigT, k);
    fT[k] = c * wT[k];
    cT[k] = c;
}

// y = x - a on the owned tree slice (forward operator u - K(sigma_s u), main.cpp:125-136)
__global__ void k_sub_slice(int64_t n, const double* __restrict__ x, const double* __restrict__ a,
                            double* __restrict__ y) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i] - a[i];
}


// Up pass (bbfmm.h:825-861) as tiers of <= 4-level subtrees:
// one workgroup per subtree keeps its nodes' multipoles in LDS, deepest level
// first; a leaf's multipole is P2M over its contiguous tree-order points
// (bbfmm.h:737-748), an internal node's is M2M of its children (bbfmm.h:855-859),
// where a child below the tier is the root of a lower tier's task (read from HBM).
// Phase 0 stages the transfer matrices, node boxes and child codes in LDS with
// one round of independent loads; the levels then run out of LDS.
// One thread per (node, entry r), r = 4j + i:  M[r] = sum_p S(x_p, c_i) S(y_p, c_j) f_p.
__global__ void __launch_bounds__(kUpThreads) k_up_tier(
    int taskBase, int maxTask, const int4* __restrict__ desc, const int* __restrict__ grpFix,
    const int* __restrict__ node, const int4* __restrict__ code, const double4* __restrict__ geom,
    const int2* __restrict__ leafRange, const double* __restrict__ pxT, const double* __restrict__ pyT,
    const double* __restrict__ xin, int treeIn, const int* __restrict__ perm, const double* __restrict__ sigT,
    const double* __restrict__ wT, double* __restrict__ fT, double* __restrict__ cT, const Params* __restrict__ P,
    double* __restrict__ mult) {
    extern __shared__ double sm[];
    int4* CD = reinterpret_cast<int4*>(sm);             // maxTask child codes
    double* Rl = reinterpret_cast<double*>(CD + maxTask);  // 4 x 256 transfer matrices (transposed)
    double* M = Rl + 4 * kRank * kRank;                 // maxTask x 16 multipoles
    double* G = M + (size_t)maxTask * kRank;            // maxTask x 4: cx, cy, 1/rx, 1/ry
    int* LB = reinterpret_cast<int*>(G + (size_t)maxTask * 4);  // maxTask: leaf point offset, count, node
    int* LC = LB + maxTask;
    int* ND = LC + maxTask;
    const int task = taskBase + blockIdx.x;
    ANISO_STAMP(0, task, 0);
    const int4 d = desc[task];  // first node, nodes, first point, levels
    const int n0 = d.x, nt = d.y, ngrp = d.w;
    const int64_t b0 = d.z;
    const int* gs = grpFix + (size_t)task * (kTaskLevels + 1);
    // M2M reads R[q][rr + 16 r] along rr: stage it transposed (r fastest) so the
    // 16 lanes of one node hit 16 consecutive LDS words
    for (int i = threadIdx.x; i < 4 * kRank * kRank; i += blockDim.x) {
        const int q = i >> 8, rr = (i >> 4) & 15, r = i & 15;
        Rl[i] = P->R[q][rr + r * kRank];
    }
    for (int k = threadIdx.x; k < nt; k += blockDim.x) {
        const double4 g = geom[n0 + k];
        G[4 * k] = g.x;
        G[4 * k + 1] = g.y;
        G[4 * k + 2] = g.z;
        G[4 * k + 3] = g.w;
        const int2 lr = leafRange[n0 + k];
        LB[k] = lr.x;
        LC[k] = lr.y;
        CD[k] = code[n0 + k];
        ND[k] = node[n0 + k];
    }
    __syncthreads();
    ANISO_STAMP(0, task, 1);
    // each point is read once (lane per point, coalesced): no LDS staging
    // P2M of the task's leaves (bbfmm.h:737-748): 16 lanes per leaf, one point per
    // lane per pass (its 16 products in registers), then a 16-lane reduce-scatter
    // leaves lane l with entry l.  The weighted charges are formed here from the
    // apply's input (the reference's charge .* weights, AnisoWrapper.cpp:105-110).
    {
        const int gi = threadIdx.x >> 4, ln = threadIdx.x & 15, ngrp = blockDim.x >> 4;
        for (int k = gi; k < nt; k += ngrp) {
            if (CD[k].x != kLeafCode) continue;  // uniform over the 16 lanes
            const double cx = G[4 * k], cy = G[4 * k + 1], irx = G[4 * k + 2], iry = G[4 * k + 3];
            const int pe = LB[k] + LC[k];
            double acc[kRank];
#pragma unroll
            for (int e = 0; e < kRank; ++e) acc[e] = 0.0;
            for (int p = LB[k] + ln; p < pe; p += 16) {
                const int64_t kp = b0 + p;
                const double c = input_charge(xin, treeIn, perm, sigT, kp);
                const double f = c * wT[kp];
                fT[kp] = f;  // for k_near and the corrections
                cT[kp] = c;
                double Sx[kNP], Sy[kNP];
                cheb_weights(P, (pxT[kp] - cx) * irx, Sx);
                cheb_weights(P, (pyT[kp] - cy) * iry, Sy);
#pragma unroll
                for (int j = 0; j < kNP; ++j) {
                    const double sf = Sy[j] * f;
#pragma unroll
                    for (int i = 0; i < kNP; ++i) acc[j * kNP + i] += Sx[i] * sf;
                }
            }
#define ANISO_RS16(NV, OFF)                                        \
    {                                                              \
        const bool hi = ln & (OFF);                                \
        _Pragma("unroll") for (int e = 0; e < (NV); ++e) {         \
            const double keep = hi ? acc[e + (NV)] : acc[e];       \
            const double send = hi ? acc[e] : acc[e + (NV)];       \
            acc[e] = keep + __shfl_xor(send, (OFF));               \
        }                                                          \
    }
            ANISO_RS16(8, 8)
            ANISO_RS16(4, 4)
            ANISO_RS16(2, 2)
            ANISO_RS16(1, 1)
#undef ANISO_RS16
            M[(size_t)k * kRank + ln] = acc[0];
        }
    }
    __syncthreads();
    ANISO_STAMP(0, task, 2);
    for (int g = 0; g < ngrp; ++g) {
        const int s0 = gs[g], s1 = gs[g + 1];
        for (int it = threadIdx.x; it < (s1 - s0) * kRank; it += blockDim.x) {
            const int k = s0 + (it >> 4), r = it & (kRank - 1);
            const int4 c = CD[k];
            double acc = 0.0;
            if (c.x == kLeafCode) continue;  // P2M above
            {
                const int cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (cs[q] == -1) continue;
                    const double* R = Rl + q * kRank * kRank + r;  // transposed: R[rr * 16 + r]
                    double a = 0.0;
                    if (cs[q] >= 0) {  // child in this task (LDS)
                        const double* cm = M + (size_t)cs[q] * kRank;
#pragma unroll
                        for (int rr = 0; rr < kRank; ++rr) a += R[rr * kRank] * cm[rr];
                    } else {  // root of the tier below (HBM)
                        const double* cm = mult + (size_t)(-cs[q] - 2) * kRank;
                        double v[kRank];
#pragma unroll
                        for (int rr = 0; rr < kRank; ++rr) v[rr] = cm[rr];
#pragma unroll
                        for (int rr = 0; rr < kRank; ++rr) a += R[rr * kRank] * v[rr];
                    }
                    acc += a;
                }
            }
            M[(size_t)k * kRank + r] = acc;
        }
        __syncthreads();
    }
    ANISO_STAMP(0, task, 3);
    for (int it = threadIdx.x; it < nt * kRank; it += blockDim.x)
        mult[(size_t)ND[it >> 4] * kRank + (it & (kRank - 1))] = M[it];
    ANISO_STAMP(0, task, 4);
}

// Lane-quad exchange through DPP quad_perm (no LDS round trip).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double quad_sum(double v) {
    v += dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
    return v;
}

// One 2 KB block as 64 lanes x 32 B: lane l reads doubles 4l .. 4l+3.  `ok`
// is wave-uniform: a skipped block reads as zeros (the predicated tail of a
// group costs no extra round trip).
__device__ __forceinline__ void load_block(const double* __restrict__ K, int64_t p, int lane, bool ok, dbl2& x0,
                                           dbl2& x1) {
    x0 = dbl2{0.0, 0.0};
    x1 = dbl2{0.0, 0.0};
    if (ok) {
        const dbl2* k = reinterpret_cast<const dbl2*>(K + (size_t)p * 256) + 2 * lane;
        x0 = __builtin_nontemporal_load(k);
        x1 = __builtin_nontemporal_load(k + 1);
    }
}

__global__ void __launch_bounds__(256) k_m2l(int ntgt, const int* __restrict__ tgt, const int64_t* __restrict__ ptr,
                                             const int* __restrict__ nDir, const int* __restrict__ canonBase,
                                             const int* __restrict__ outSlot, const int* __restrict__ src,
                                             const double* __restrict__ K, const double* __restrict__ mult, double sgn,
                                             double* __restrict__ partial, double* __restrict__ local) {
    // wave-uniform indexing (readfirstlane): descriptors and source ids come
    // through the scalar unit, so the stream's addresses never wait on a load
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) / kWave));
    const int lane = threadIdx.x & (kWave - 1);
    if (wave >= ntgt) return;
    const int n = tgt[wave];
    const int t = lane >> 2, q = lane & 3;
    const int64_t p0 = ptr[wave], p1 = ptr[wave + 1], pd = p0 + nDir[wave];
    const int nC = (int)(p1 - pd);  // canonical pairs, <= kMaxCanon (host plan)
    // lane-parallel prefetch of the canonical sources and their partial slots
    const int cSrc = lane < nC ? src[pd + lane] : 0;
    const int cSlot = lane < nC ? outSlot[canonBase[wave] + lane] : 0;
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    // ---- directed pairs (row-major): lane owns row t, columns 4q .. 4q+3
    for (int64_t c = p0; c < pd; c += kWave) {
        const int cnt = (int)min<int64_t>(kWave, pd - c);
        const int mySrc = lane < cnt ? src[c + lane] : 0;
        for (int j = 0; j < cnt; j += 4) {
            dbl2 a0, a1, b0, b1, c0, c1, d0, d1;
            load_block(K, c + j, lane, true, a0, a1);
            load_block(K, c + j + 1, lane, j + 1 < cnt, b0, b1);
            load_block(K, c + j + 2, lane, j + 2 < cnt, c0, c1);
            load_block(K, c + j + 3, lane, j + 3 < cnt, d0, d1);
            // a skipped block's source id is a valid clamp; its block is zero
            const double4 ma = *reinterpret_cast<const double4*>(mult + (size_t)__builtin_amdgcn_readlane(mySrc, j) * kRank + q * 4);
            const double4 mb = *reinterpret_cast<const double4*>(mult + (size_t)__builtin_amdgcn_readlane(mySrc, min(j + 1, cnt - 1)) * kRank + q * 4);
            const double4 mc = *reinterpret_cast<const double4*>(mult + (size_t)__builtin_amdgcn_readlane(mySrc, min(j + 2, cnt - 1)) * kRank + q * 4);
            const double4 md = *reinterpret_cast<const double4*>(mult + (size_t)__builtin_amdgcn_readlane(mySrc, min(j + 3, cnt - 1)) * kRank + q * 4);
            acc0 += a0.x * ma.x + a0.y * ma.y + a1.x * ma.z + a1.y * ma.w;
            acc1 += b0.x * mb.x + b0.y * mb.y + b1.x * mb.z + b1.y * mb.w;
            acc2 += c0.x * mc.x + c0.y * mc.y + c1.x * mc.z + c1.y * mc.w;
            acc3 += d0.x * md.x + d0.y * md.y + d1.x * md.z + d1.y * md.w;
        }
    }
    double acc = (acc0 + acc1) + (acc2 + acc3);
    // ---- canonical pairs (column-major): lane owns column s = t, rows 4q .. 4q+3
    if (nC > 0) {
        const double4 mn = *reinterpret_cast<const double4*>(mult + (size_t)n * kRank + q * 4);
        const double m0 = sgn * mn.x, m1 = sgn * mn.y, m2 = sgn * mn.z, m3 = sgn * mn.w;
        double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;  // forward rows 4q+j, this lane's column
        // transposed products stay in registers (lane (s, q) keeps entry s of pair
        // 4g + q) and are stored after the stream: on CDNA vmcnt also counts
        // stores, so stores inside the loop would stall it
        constexpr int kGroups = (kMaxCanon + 3) / 4;
        double y[kGroups];
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
            y[g] = 0.0;
            const int j = 4 * g;
            if (j < nC) {
                dbl2 a0, a1, b0, b1, e0, e1, f0, f1;
                load_block(K, pd + j, lane, true, a0, a1);
                load_block(K, pd + j + 1, lane, j + 1 < nC, b0, b1);
                load_block(K, pd + j + 2, lane, j + 2 < nC, e0, e1);
                load_block(K, pd + j + 3, lane, j + 3 < nC, f0, f1);
                const double xa = mult[(size_t)__builtin_amdgcn_readlane(cSrc, j) * kRank + t];
                const double xb = mult[(size_t)__builtin_amdgcn_readlane(cSrc, min(j + 1, nC - 1)) * kRank + t];
                const double xe = mult[(size_t)__builtin_amdgcn_readlane(cSrc, min(j + 2, nC - 1)) * kRank + t];
                const double xf = mult[(size_t)__builtin_amdgcn_readlane(cSrc, min(j + 3, nC - 1)) * kRank + t];
                c0 += (a0.x * xa + b0.x * xb) + (e0.x * xe + f0.x * xf);
                c1 += (a0.y * xa + b0.y * xb) + (e0.y * xe + f0.y * xf);
                c2 += (a1.x * xa + b1.x * xb) + (e1.x * xe + f1.x * xf);
                c3 += (a1.y * xa + b1.y * xb) + (e1.y * xe + f1.y * xf);
                const double ya = quad_sum(a0.x * m0 + a0.y * m1 + a1.x * m2 + a1.y * m3);
                const double yb = quad_sum(b0.x * m0 + b0.y * m1 + b1.x * m2 + b1.y * m3);
                const double ye = quad_sum(e0.x * m0 + e0.y * m1 + e1.x * m2 + e1.y * m3);
                const double yf = quad_sum(f0.x * m0 + f0.y * m1 + f1.x * m2 + f1.y * m3);
                y[g] = q == 0 ? ya : q == 1 ? yb : q == 2 ? ye : yf;
            }
        }
        // partial slots: lane (s, q) stores entry s of pair 4g + q (8 B lanes, 128 B
        // per pair); slot ids shuffled with every lane active
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
            if (4 * g < nC) {
                const int jj = 4 * g + q;
                const int slot = __shfl(cSlot, jj);
                if (jj < nC) partial[(size_t)slot * kRank + t] = y[g];
            }
        }
        // forward rows: sum c_j over the 16 columns (lane bits 2..5), then row
        // t = 4q' + j sits in entry j of the lanes with q == q' (e.g. lane q')
#pragma unroll
        for (int off = 4; off < kWave; off <<= 1) {
            c0 += __shfl_xor(c0, off);
            c1 += __shfl_xor(c1, off);
            c2 += __shfl_xor(c2, off);
            c3 += __shfl_xor(c3, off);
        }
        const int jr = t & 3;
        const double v = jr == 0 ? c0 : jr == 1 ? c1 : jr == 2 ? c2 : c3;  // row 4q + jr
        // lane (t, q) needs row t = 4(t>>2) + jr from a lane with q == t>>2
        const double w = __shfl(v, 4 * t + (t >> 2));
        if (q == 0) acc += w;
    }
    acc = quad_sum(acc);
    if (q == 0) local[(size_t)n * kRank + t] = acc;
}

// local[B] += the transposed canonical-pair products addressed to B: one
// contiguous slot range per target, summed in a fixed order (deterministic).
// One thread per (target, entry); 8 independent loads in flight per thread.
__global__ void __launch_bounds__(256) k_m2l_gather(int ntgt, const int* __restrict__ tgt, const int* __restrict__ inPtr,
                                                    const double* __restrict__ partial, double* __restrict__ local) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int w = gid >> 4, r = gid & 15;
    if (w >= ntgt) return;
    const int j0 = inPtr[w], j1 = inPtr[w + 1];
    if (j0 == j1) return;
    const double* pp = partial + (size_t)j0 * kRank + r;
    const int n = j1 - j0;
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int j = 0;
    for (; j + 7 < n; j += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += __builtin_nontemporal_load(pp + (size_t)(j + u) * kRank);
    }
#pragma unroll
    for (int u = 0; u < 7; ++u)
        if (j + u < n) a[u] += __builtin_nontemporal_load(pp + (size_t)(j + u) * kRank);
    local[(size_t)tgt[w] * kRank + r] += ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// U/W near field for one target leaf per wave (bbfmm.h:1081-1099, 1111-1113).
// All per-leaf indexing comes from host-built descriptors loaded lane-parallel,
// so a wave pays ~3 memory round trips before it starts streaming its block:
//   leafInfo[li] = (node, begin, count, S), nearPts = the S source tree positions
//   leafChain    = the leaf's ancestors from level 1 down to the leaf itself.
// The block is column-major nTs x S (rows padded to even nTs): each lane reads
// 16 B = two targets of one source column; lanes = (row pair, column phase),
// 4 independent loads in flight per lane.
__global__ void __launch_bounds__(256) k_near(int nl, const int4* __restrict__ leafInfo,
                                              const int64_t* __restrict__ nearPtsPtr, const int* __restrict__ nearPts,
                                              const int64_t* __restrict__ nearKOff, const int2* __restrict__ nearSym,
                                              const double* __restrict__ K, const double* __restrict__ fT,
                                              const int* __restrict__ operm, int64_t obase, int maxS, int flags,
                                              double sgn, double scale, double* __restrict__ partial,
                                              double* __restrict__ out) {
    extern __shared__ double sh[];
    const int wv = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    const int li = blockIdx.x * (blockDim.x / kWave) + wv;
    const bool active = li < nl;
    double* fs = sh + (size_t)wv * maxS;
    int4 info = make_int4(0, 0, 0, 0);
    int64_t koff = 0;
    if (active) {
        info = leafInfo[li];
        const int64_t pb = nearPtsPtr[li];
        koff = nearKOff[li];
        // stage the S source charges (lane-parallel gather, 4 loads in flight per lane)
        const int S = info.w;
        for (int s0 = 0; s0 < S; s0 += 4 * kWave) {
            int ix[4];
            double fv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int sidx = s0 + u * kWave + lane;
                ix[u] = sidx < S ? nearPts[pb + sidx] : -1;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) fv[u] = ix[u] >= 0 ? fT[ix[u]] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int sidx = s0 + u * kWave + lane;
                if (sidx < S) fs[sidx] = fv[u];
            }
        }
    }
    __syncthreads();
    if (!active) return;
    const int nT = info.z, S = info.w;
    const int2 sym = nearSym[li];  // (directed source points Sdir, partial base)
    const int Sdir = sym.x;
    const int64_t tb = info.y;
    const double* Kl = K + koff;
    const int nTs = nT + (nT & 1);
    const int rp = nTs >> 1;
    int lpc = 1;
    while (lpc < rp && lpc < kWave) lpc <<= 1;
    const int cps = kWave / lpc;
    const int cph = lane / lpc;
    for (int rc = 0; rc < rp; rc += kWave) {
        const int r = rc + (lane & (lpc - 1));
        double a0 = 0.0, a1 = 0.0;
        if ((flags & kStageNear) && S > Sdir) {
            // canonical U pairs (host: only when rp <= 64): one read of each column
            // gives this leaf's row sums and the other leaf's transposed product
            // sgn * sum_t K[t][s] f[t], reduced over the column's lanes.
            const dbl2* kc = reinterpret_cast<const dbl2*>(Kl) + r;
            const double fa0 = (r < rp && 2 * r < nT) ? fT[tb + 2 * r] : 0.0;
            const double fa1 = (r < rp && 2 * r + 1 < nT) ? fT[tb + 2 * r + 1] : 0.0;
            const int ncol = S - Sdir;
            for (int i0 = 0; i0 < ncol; i0 += 4 * cps) {  // 4 columns per lane in flight
                dbl2 kk[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int s = Sdir + i0 + u * cps + cph;
                    ok[u] = (i0 + u * cps + cph < ncol) && r < rp;
                    kk[u] = ok[u] ? __builtin_nontemporal_load(kc + (size_t)s * rp) : dbl2{0.0, 0.0};
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int s = Sdir + i0 + u * cps + cph;
                    const double fsv = ok[u] ? fs[s] : 0.0;
                    a0 += kk[u].x * fsv;
                    a1 += kk[u].y * fsv;
                    double c = kk[u].x * fa0 + kk[u].y * fa1;
                    for (int off = 1; off < lpc; off <<= 1) c += __shfl_xor(c, off);
                    // column s's charge is consumed: its LDS word now holds the
                    // product, stored after the stream (vmcnt also counts stores)
                    if (ok[u] && (lane & (lpc - 1)) == 0) fs[s] = sgn * c;
                }
            }
        }
        if ((flags & kStageNear) && r < rp) {
            const dbl2* kc = reinterpret_cast<const dbl2*>(Kl) + r;
            const int stride = rp;  // dbl2 elements per column
            int s = cph;
            const int S = Sdir;  // directed columns
            for (; s + 3 * cps < S; s += 4 * cps) {
                dbl2 k0 = __builtin_nontemporal_load(kc + (size_t)s * stride);
                dbl2 k1 = __builtin_nontemporal_load(kc + (size_t)(s + cps) * stride);
                dbl2 k2 = __builtin_nontemporal_load(kc + (size_t)(s + 2 * cps) * stride);
                dbl2 k3 = __builtin_nontemporal_load(kc + (size_t)(s + 3 * cps) * stride);
                double f0 = fs[s], f1 = fs[s + cps], f2 = fs[s + 2 * cps], f3 = fs[s + 3 * cps];
                a0 += k0.x * f0 + k1.x * f1 + k2.x * f2 + k3.x * f3;
                a1 += k0.y * f0 + k1.y * f1 + k2.y * f2 + k3.y * f3;
            }
            for (; s < S; s += cps) {
                dbl2 k0 = __builtin_nontemporal_load(kc + (size_t)s * stride);
                a0 += k0.x * fs[s];
                a1 += k0.y * fs[s];
            }
        }
        for (int off = lpc; off < kWave; off <<= 1) {
            a0 += __shfl_xor(a0, off);
            a1 += __shfl_xor(a1, off);
        }
        if (cph == 0 && r < rp) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int t = 2 * r + h;
                if (t >= nT) break;
                out[out_index(operm, obase, tb + t)] = scale * (h ? a1 : a0);
            }
        }
    }
    if ((flags & kStageNear) && S > Sdir) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int i = lane; i < S - Sdir; i += kWave) partial[(int64_t)sym.y + i] = fs[Sdir + i];
    }
}

// Down pass (bbfmm.h:1066-1106) as tiers of <= 4-level subtrees, top-down, after
// k_m2l, k_m2l_gather and k_near.  Per node: total = local (its M2L, transposed
// partials included) + L2L of the parent's total
// (bbfmm.h:1070-1071; the parent is in LDS, or in HBM for a task root).  Then per
// owned leaf point: L2P (bbfmm.h:1104) + the gathered transposed U-pair products
// of k_near, added to out.  dn = (node, parent code, child slot, 0).
// Phase 0 issues every independent global load of the task at once (locals of
// all nodes, the roots' parent totals, box geometry, points and
// their output slots) into LDS; the levels and the points then run out of LDS.
__global__ void __launch_bounds__(kTierThreads) k_down_tier(
    int maxTask, int maxLeaves, const int4* __restrict__ desc, const int* __restrict__ grpFix,
    const int4* __restrict__ dn, const double* __restrict__ local, const Params* __restrict__ P,
    const int* __restrict__ leafSlot, const int* __restrict__ leafBegin, const int2* __restrict__ leafNear,
    const double4* __restrict__ leafGeom, const double* __restrict__ pxT, const double* __restrict__ pyT,
    const int* __restrict__ operm, int64_t obase, const int* __restrict__ nearOff, int maxNear,
    const double* __restrict__ nearPart, const int2* __restrict__ chain, int maxChain, int flags, double scale,
    double* __restrict__ out) {
    extern __shared__ double sm[];
    int4* DN = reinterpret_cast<int4*>(sm);             // maxTask node records
    double* Rl = reinterpret_cast<double*>(DN + maxTask);  // 4 x 256 transfer matrices
    double* T = Rl + 4 * kRank * kRank;                 // maxTask x 16 totals
    double* PT = T + (size_t)maxTask * kRank;           // 16: the task root's parent total
    double* CH = PT + kRank;                            // maxChain x 16: the ancestors' locals
    double* G = CH + (size_t)maxChain * kRank;          // maxLeaves x 4: leaf cx, cy, 1/rx, 1/ry
    int* LB = reinterpret_cast<int*>(G + (size_t)maxLeaves * 4);  // maxLeaves + 1: leaf begins (tree positions)
    int* LS = LB + maxLeaves + 1;                       // maxLeaves: leaf slot in the task
    int* NB = LS + maxLeaves;                           // maxLeaves: first of the leaf's near offsets in NO
    int* NC = NB + maxLeaves;                           // maxLeaves: their count
    int* NO = NC + maxLeaves;                           // maxNear: partial offsets of the blocks addressed here
    const int task = blockIdx.x;
    ANISO_STAMP(1, task, 0);
    // task record: (first node, nodes, first leaf entry, leaves), (owned points begin,
    // end, first chain entry, chain length), (first near offset, count, levels, 0)
    const int4 d0 = desc[3 * task], d1 = desc[3 * task + 1], d2 = desc[3 * task + 2];
    const int n0 = d0.x, nt = d0.y, l0 = d0.z, nl = d0.w;
    const int2 pr = make_int2(d1.x, d1.y);
    const int c0 = d1.z, nc = d1.w;
    const int npts = pr.y - pr.x, ngrp = d2.z;
    const int* gs = grpFix + (size_t)task * (kTaskLevels + 1);
    const bool far = flags & kStageFar;
    // ---- phase 0: independent loads
    if (far) {
        for (int i = threadIdx.x; i < 4 * kRank * kRank; i += blockDim.x) Rl[i] = (&P->R[0][0])[i];
        for (int k = threadIdx.x; k < nt; k += blockDim.x) DN[k] = dn[n0 + k];
        for (int it = threadIdx.x; it < nt * kRank; it += blockDim.x) {
            const int k = it >> 4, r = it & (kRank - 1);
            T[it] = local[(size_t)dn[n0 + k].x * kRank + r];
        }
        for (int it = threadIdx.x; it < nc * kRank; it += blockDim.x)
            CH[it] = local[(size_t)chain[c0 + (it >> 4)].x * kRank + (it & (kRank - 1))];
    }
    for (int e = threadIdx.x; e < nl; e += blockDim.x) {
        LB[e] = leafBegin[l0 + e];
        LS[e] = leafSlot[l0 + e];
        const int2 ni = leafNear[l0 + e];
        NB[e] = ni.x;
        NC[e] = ni.y;
        const double4 g = leafGeom[l0 + e];
        G[4 * e] = g.x;
        G[4 * e + 1] = g.y;
        G[4 * e + 2] = g.z;
        G[4 * e + 3] = g.w;
    }
    if (threadIdx.x == 0) LB[nl] = pr.y;
    for (int j = threadIdx.x; j < d2.y; j += blockDim.x) NO[j] = nearOff[d2.x + j];
    __syncthreads();
    ANISO_STAMP(1, task, 1);
    // ---- phase 1: the root's parent total by the L2L chain from level 1 (one
    // 16-lane group; bbfmm.h:1070-1071 along the ancestors), then the task's levels
    if (far) {
        if (threadIdx.x < kRank) {
            const int r = threadIdx.x;
            double v = nc > 0 ? CH[r] : 0.0;
            for (int j = 1; j < nc; ++j) {
                const double* R = Rl + chain[c0 + j].y * kRank * kRank;
                double a = CH[j * kRank + r];
#pragma unroll
                for (int c = 0; c < kRank; ++c) a += R[r + c * kRank] * __shfl(v, c, kRank);
                v = a;
            }
            PT[r] = v;
        }
        __syncthreads();
        ANISO_STAMP(1, task, 2);
        for (int g = 0; g < ngrp; ++g) {
            const int s0 = gs[g], s1 = gs[g + 1];
            for (int it = threadIdx.x; it < (s1 - s0) * kRank; it += blockDim.x) {
                const int k = s0 + (it >> 4), r = it & (kRank - 1);
                const int4 d = DN[k];
                if (d.y == -1) continue;
                const double* pt = d.y >= 0 ? T + (size_t)d.y * kRank : PT;  // -2: the task root
                const double* R = Rl + d.z * kRank * kRank;
                double l2l = 0.0;
#pragma unroll
                for (int c = 0; c < kRank; ++c) l2l += R[r + c * kRank] * pt[c];
                T[(size_t)k * kRank + r] += l2l;
            }
            __syncthreads();
        }
    }
    ANISO_STAMP(1, task, 3);
    // ---- phase 2: owned points: L2P + near gather
    for (int g = threadIdx.x; g < npts; g += blockDim.x) {
        const int kpos = pr.x + g;
        int lo = 0, hi = nl - 1;  // last leaf with LB <= kpos
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (LB[mid] <= kpos) lo = mid;
            else hi = mid - 1;
        }
        const int t = kpos - LB[lo];
        double v = 0.0;
        if (flags & kStageNear) {
            const int* no = NO + NB[lo];
            for (int j = 0; j < NC[lo]; ++j) v += nearPart[(size_t)no[j] + t];
        }
        if (far) {
            const double x = pxT[kpos], y = pyT[kpos];
            double Sx[kNP], Sy[kNP];
            cheb_weights(P, (x - G[4 * lo]) * G[4 * lo + 2], Sx);
            cheb_weights(P, (y - G[4 * lo + 1]) * G[4 * lo + 3], Sy);
            const double* L = T + (size_t)LS[lo] * kRank;
            double l2p = 0.0;
#pragma unroll
            for (int j = 0; j < kNP; ++j)
#pragma unroll
                for (int i = 0; i < kNP; ++i) l2p += Sx[i] * Sy[j] * L[j * kNP + i];
            v += l2p;
        }
        out[out_index(operm, obase, kpos)] += scale * v;
    }
    ANISO_STAMP(1, task, 4);
}

// Corrections (nearRemoval + refineAddOnFast + singularAddFast,
// KernelFactory.cpp:445-478, 662-709, 828-860) as a 3x3-square stencil with
// per-mode translation-invariant d2 x 9 x d2 weights, plus the singular term
// from Legendre coefficients of the target's own square (O(d^4) moments).  Every
// contribution carries the final 1/(2 pi) (AnisoWrapper.cpp:129-130): k_near
// stores its scaled sum, k_corr and k_down_tier add theirs, in any order.
template <int D>
__global__ void __launch_bounds__(256) k_corr(int64_t b, int64_t e, const int* __restrict__ perm,
                                              const int* __restrict__ iperm, const double* __restrict__ cT,
                                              const double* __restrict__ fT,
                                              const double* __restrict__ C, const double* __restrict__ mu,
                                              const Params* __restrict__ P, int flags, double scale,
                                              bool treeOut, double* __restrict__ out) {
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
                const int* it = iperm + (size_t)(sq + dr * sz + dc) * D2;  // the square's points, tree positions
#pragma unroll
                for (int c = 0; c < D2; ++c) acc += w[c] * fT[it[c]];
            }
        }
    }
    if (flags & kStageSing) {
        const int* it = iperm + (size_t)sq * D2;
        double hw[D2];
#pragma unroll
        for (int c = 0; c < D2; ++c) hw[c] = P->sqrtW[c] * cT[it[c]];
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
    out[treeOut ? k - b : (int64_t)t] += acc * scale;  // near and far are scaled by their own kernels
}

__global__ void k_permute(int64_t N, const int* __restrict__ perm, const double* __restrict__ orig,
                          double* __restrict__ tree) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) tree[k] = orig[perm[k]];
}

// ----------------------------------------------------------------- cache build

// downPassCache's M2L blocks (bbfmm.h:959-975, 782-804) for all stored (target,
// source) pairs, K[t][s] = kernel(cheb_s(src), cheb_t(tgt)): directed blocks
// row-major (pair*256 + t*16 + s), canonical blocks (pairTgt = ~target)
// column-major (pair*256 + s*16 + t), the layouts k_m2l streams.
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
    if (tn < 0) {  // canonical: column-major
        tn = ~tn;
        const int tmp = t;
        t = s;
        s = tmp;
    }
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
    const int nTs = nT + (nT & 1);  // rows padded to even (16-B loads in k_near)
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

static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

void launch_prepare(int64_t N, const double* xin, int treeIn, const int* perm, const double* sigT, const double* wT,
                    double* fT, double* cT, hipStream_t s) {
    if (N <= 0) return;
    k_prepare<<<blocks_for(N, 256), 256, 0, s>>>(N, xin, treeIn, perm, sigT, wT, fT, cT);
    HIP_LAUNCH_CHECK();
}

size_t up_tier_lds(int maxTask) {
    return (size_t)(4 * kRank * kRank + maxTask * (kRank + 4)) * sizeof(double) + (size_t)3 * maxTask * sizeof(int) +
           (size_t)maxTask * sizeof(int4);
}

size_t down_tier_lds(int maxTask, int maxLeaves, int maxNear, int maxChain) {
    return (size_t)(4 * kRank * kRank + maxTask * kRank + kRank + maxChain * kRank + 4 * maxLeaves) * sizeof(double) +
           (size_t)(4 * maxLeaves + 4 + maxNear) * sizeof(int) + (size_t)maxTask * sizeof(int4);
}

void launch_up_tier(int ntask, int taskBase, int maxTask, const int4* desc, const int* grpFix, const int* node,
                    const int4* code, const double4* geom, const int2* leafRange, const double* pxT, const double* pyT,
                    const double* xin, int treeIn, const int* perm, const double* sigT, const double* wT, double* fT,
                    double* cT, const Params* P, double* mult, hipStream_t s) {
    if (ntask <= 0) return;
    k_up_tier<<<ntask, kUpThreads, up_tier_lds(maxTask), s>>>(taskBase, maxTask, desc, grpFix, node, code, geom,
                                                               leafRange, pxT, pyT, xin, treeIn, perm, sigT, wT, fT,
                                                               cT, P, mult);
    HIP_LAUNCH_CHECK();
}

void launch_m2l(int ntgt, const int* tgt, const int64_t* ptr, const int* nDir, const int* canonBase,
                const int* outSlot, const int* src, const double* K, const double* mult, double sgn, double* partial,
                double* local, hipStream_t s) {
    if (ntgt <= 0) return;
    k_m2l<<<blocks_for((int64_t)ntgt * kWave, 256), 256, 0, s>>>(ntgt, tgt, ptr, nDir, canonBase, outSlot, src, K, mult,
                                                                sgn, partial, local);
    HIP_LAUNCH_CHECK();
}

void launch_m2l_gather(int ntgt, const int* tgt, const int* inPtr, const double* partial, double* local,
                       hipStream_t s) {
    if (ntgt <= 0) return;
    k_m2l_gather<<<blocks_for((int64_t)ntgt * kRank, 256), 256, 0, s>>>(ntgt, tgt, inPtr, partial, local);
    HIP_LAUNCH_CHECK();
}

void launch_near(int nl, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts, const int64_t* nearKOff,
                 const int2* nearSym, const double* K, const double* fT, const int* operm, int64_t obase, int maxS,
                 int flags, double sgn, double scale, double* partial, double* out, hipStream_t s) {
    if (nl <= 0) return;
    int wpb = maxS * 8 * 4 <= 48 * 1024 ? 4 : 1;
    size_t shm = (size_t)wpb * (maxS > 0 ? maxS : 1) * sizeof(double);
    k_near<<<blocks_for(nl, wpb), wpb * kWave, shm, s>>>(nl, leafInfo, nearPtsPtr, nearPts, nearKOff, nearSym, K, fT,
                                                        operm, obase, maxS > 0 ? maxS : 1, flags, sgn, scale,
                                                        partial, out);
    HIP_LAUNCH_CHECK();
}

void launch_down_tier(int ntask, int maxTask, int maxLeaves, const int4* desc, const int* grpFix, const int4* dn,
                      const double* local, const Params* P, const int* leafSlot, const int* leafBegin,
                      const int2* leafNear, const double4* leafGeom, const double* pxT, const double* pyT,
                      const int* operm, int64_t obase, const int* nearOff, int maxNear, const double* nearPart,
                      const int2* chain, int maxChain, int flags, double scale, double* out, hipStream_t s) {
    if (ntask <= 0) return;
    k_down_tier<<<ntask, kTierThreads, down_tier_lds(maxTask, maxLeaves, maxNear, maxChain), s>>>(
        maxTask, maxLeaves, desc, grpFix, dn, local, P, leafSlot, leafBegin, leafNear, leafGeom, pxT, pyT, operm,
        obase, nearOff, maxNear, nearPart, chain, maxChain, flags, scale, out);
    HIP_LAUNCH_CHECK();
}

void launch_corr(int d, int64_t b, int64_t e, const int* perm, const int* iperm, const double* cT, const double* fT,
                 const double* C,
                 const double* mu, const Params* P, int flags, double scale, bool treeOut, double* out,
                 hipStream_t s) {
    if (e <= b) return;
    unsigned nb = blocks_for(e - b, 256);
    switch (d) {
        case 1: k_corr<1><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, C, mu, P, flags, scale, treeOut, out); break;
        case 2: k_corr<2><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, C, mu, P, flags, scale, treeOut, out); break;
        case 3: k_corr<3><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, C, mu, P, flags, scale, treeOut, out); break;
        case 4: k_corr<4><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, C, mu, P, flags, scale, treeOut, out); break;
        case 5: k_corr<5><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, C, mu, P, flags, scale, treeOut, out); break;
        case 6: k_corr<6><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, C, mu, P, flags, scale, treeOut, out); break;
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


void launch_sub_slice(int64_t n, const double* x, const double* a, double* y, hipStream_t s) {
    if (n <= 0) return;
    k_sub_slice<<<blocks_for(n, 256), 256, 0, s>>>(n, x, a, y);
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
