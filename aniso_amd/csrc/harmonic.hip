// harmonic.hip -- the mode-shared ("harmonic") block apply of aniso.m's operator:
// all 2 nb - 1 Fourier modes of the block matvec from ONE read of a
// mode-independent cache.
//
// Reference behaviour (file:line under lowrank/aniso):
//   block caller  aniso.m:139-157   out_iid = sum_j chi_|j| K_|iid+j| (sigma_s u_|j|)
//   kernels       KernelFactory.cpp:240-267   K_m = e^-tau cos(m theta) / r (merged)
//   M2L / near    bbfmm.h:1051-1065, 1081-1099
//
// The identity.  Every mode's merged kernel is K_m(t <- s) = E(t, s) cos(m theta) / r
// with E = e^-tau(s, t) independent of m.  aniso.m's output block iid sums, over
// j in [-(nb-1), nb-1], the weight w_|j| times K_|iid+j| applied to block |j|.
// cos is even, so cos(|iid + j| theta) = cos(iid theta) cos(j theta) -
// sin(iid theta) sin(j theta), and the sine part cancels between j and -j (its
// weight and block are even in j).  Hence, per matrix entry,
//
//     sum_j w_|j| K_|iid+j|(t,s) x_|j|(s) = (E/r) cos(iid theta) V(t,s),
//     V(t,s) = sum_b hw_b cos(b theta) x_b(s),   hw_0 = w_0, hw_b = 2 w_b,
//
// with cos(b theta) = T_b(c), c = dx / r (Chebyshev recurrence).  The 45
// mode-applies of one block matvec become one pass over E (8 B per directed
// entry, shared by all modes) at ~K + 10 FMAs per entry.  At r = 0 (a point's own
// entry of the near field) only mode 0 has a value, sigma_t (KernelFactory.cpp:260):
// its term dw_iid sigma_t f_iid (dw_iid = the mode-0 weight of block iid) is added
// apart.  The host checks that the mixes have this structure (Operator::applyBlock).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "corr_point.hpp"
#include "device_common.hpp"
#include "up_task.hpp"

namespace aniso {

// 1/sqrt(x) to full double precision: v_rsq_f64 (about 2^-22 relative) and two
// Newton steps.  x = 0 gives a non-finite value; callers select it away.
__device__ __forceinline__ double rsqrt_f64(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double h = x * y;
    double e = __builtin_fma(-h, y, 1.0);
    y = __builtin_fma(0.5 * y, e, y);
    h = x * y;
    e = __builtin_fma(-h, y, 1.0);
    return __builtin_fma(0.5 * y, e, y);
}

// NR Newton steps after v_rsq_f64: one step leaves a relative error of about
// 1.5 eps0^2 (eps0 ~ 2^-22 for v_rsq_f64), i.e. ~1e-13 per kernel entry, far inside
// the 1e-10 parity tolerance; two steps give full double precision.
template <int NR>
__device__ __forceinline__ double rsqrt_nr(double x) {
    if constexpr (NR >= 2) {
        return rsqrt_f64(x);
    } else {
        const double y = __builtin_amdgcn_rsq(x);
        const double e = __builtin_fma(-(x * y), y, 1.0);
        return __builtin_fma(0.5 * y, e, y);
    }
}

// a wave-uniform double in SGPRs.  Loop-invariant table values (the Chebyshev nodes)
// read through a generic pointer are re-loaded inside loops that also do atomics on
// generic pointers (no hoisting across a possible alias); such a reload issued after a
// prefetch makes the compiler's vmcnt wait drain the prefetch as well.
__device__ __forceinline__ double uniform_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// XCD-aware workgroup order: the dispatcher deals workgroups round-robin over the
// 8 XCDs (bid % 8), so consecutive logical tiles would land on 8 different L2s.
// Renumber so each XCD runs one contiguous range of logical workgroups: targets
// in tree order are spatial neighbours and share source multipoles (and stored
// blocks read by both ends) through that XCD's L2.
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
    const int x = bid & 7, per = nb >> 3, rem = nb & 7, j = bid >> 3;
    return x < rem ? x * (per + 1) + j : rem * (per + 1) + (x - rem) * per + j;
}

// T_0 .. T_{K-1} at c (cos(b theta) for c = cos theta)
template <int K>
__device__ __forceinline__ void cheb_T(double c, double (&T)[K]) {
    T[0] = 1.0;
    if constexpr (K > 1) T[1] = c;
    const double c2 = c + c;
#pragma unroll
    for (int i = 2; i < K; ++i) T[i] = __builtin_fma(c2, T[i - 1], -T[i - 2]);
}

// One entry: E at (dx, dy) from the source, harmonic-weighted source charges xw;
// o[i] += T_i(c) (E / r) V.  guard0: r = 0 possible (near field): r^2 is raised to
// 1e-300 there, so 1/r stays finite and the entry adds exactly 0 through E = 0 (the
// mode-shared cache stores 0 at r = 0, kernels.hip pair_kernel): one v_max_f64
// instead of a compare and two selects per entry, the same bits elsewhere.
template <int K, bool guard0, int NR = 2>
__device__ __forceinline__ void hm_entry(double e, double dx, double dy2, const double (&xw)[K], double (&o)[K]) {
    double r2 = __builtin_fma(dx, dx, dy2);
    if constexpr (guard0) r2 = __builtin_fmax(r2, 1e-300);
    const double ri = rsqrt_nr<NR>(r2);
    const double c = dx * ri;
    double T[K];
    cheb_T<K>(c, T);
    double v = xw[0];
#pragma unroll
    for (int b = 1; b < K; ++b) v = __builtin_fma(T[b], xw[b], v);
    const double av = (e * ri) * v;
#pragma unroll
    for (int i = 0; i < K; ++i) o[i] = __builtin_fma(T[i], av, o[i]);
}

// ----------------------------------------------------------------- M2L

// M2L over V then X (bbfmm.h:1051-1065) for every mode of the block matvec: one
// wave per target node, every directed pair's 2 KB E block read once as 64 lanes
// x 32 B (column-major: lane (s, q) holds column s, rows 4q..4q+3); the lane's
// target rows are the Chebyshev points (x_j, y_q) of the target, its column the
// point s of the source (kernels.hip k_cache_att_m2l); PG blocks in flight.
// local[n][t][i] = sum over pairs of sum_s (E/r) T_i V (the unscaled locals of all
// output blocks; L2L / L2P in k_down_tier are mode-independent).
// Symmetric storage: a V pair whose ends are both targets here has one stored
// block (its smaller id's orientation); blk >= 0 reads block blk as stored, ~blk
// reads it transposed (E(t, s) = E_stored(s, t): tau is symmetric), lane (s, q)
// then loading rows 4q..4q+3 of its column with stride 16 (each of the 4 loads
// covers four 128-B lines across the wave).  Plain loads: the partner's read of a
// shared block should find it in the Infinity Cache.
template <int K, int PG, int NR, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) k_m2l_hm(int ntgt, int xcd, const int* __restrict__ tgt,
                                                const int64_t* __restrict__ ptr, const int* __restrict__ src,
                                                const int* __restrict__ blk,
                                                const double* __restrict__ E, const double* __restrict__ ncx,
                                                const double* __restrict__ ncy, const double* __restrict__ nrx,
                                                const double* __restrict__ nry, const Params* __restrict__ P,
                                                HarmWeights hw, const double* __restrict__ mult,
                                                double* __restrict__ local) {
    const int bid = xcd ? xcd_tile((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(bid * (int)(blockDim.x / kWave) + (int)(threadIdx.x / kWave));
    const int lane = threadIdx.x & (kWave - 1);
    if (wave >= ntgt) return;
    const int n = tgt[wave];
    const int s = lane >> 2, q = lane & 3;
    double bx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bx[j] = ncx[n] + nrx[n] * P->cheb[j];
    const double by = ncy[n] + nry[n] * P->cheb[q];
    const double chx = P->cheb[s & 3], chy = P->cheb[s >> 2];
    double c[4][K];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < K; ++i) c[j][i] = 0.0;
    const int64_t p0 = ptr[wave], p1 = ptr[wave + 1];
    for (int64_t cb = p0; cb < p1; cb += kWave) {
        const int cnt = (int)min<int64_t>(kWave, p1 - cb);
        const int mySrc = lane < cnt ? src[cb + lane] : 0;
        const int myBlk = lane < cnt ? blk[cb + lane] : 0;
        for (int j0 = 0; j0 < cnt; j0 += PG) {
            double e4[PG][4];
            double xm[PG][K];
            int B[PG];
#pragma unroll
            for (int g = 0; g < PG; ++g) {
                const int b = __builtin_amdgcn_readlane(myBlk, min(j0 + g, cnt - 1));
                const bool tr = b < 0;
                const double* p = E + (size_t)(tr ? ~b : b) * 256 + (tr ? 64 * q + s : 16 * s + 4 * q);
                const int st = tr ? 16 : 1;
#pragma unroll
                for (int j = 0; j < 4; ++j) e4[g][j] = j0 + g < cnt ? p[j * st] : 0.0;
            }
#pragma unroll
            for (int g = 0; g < PG; ++g) {  // a skipped block's source is a valid clamp; its E is zero
                B[g] = __builtin_amdgcn_readlane(mySrc, min(j0 + g, cnt - 1));
                const double* m = mult + ((size_t)B[g] * kRank + s) * K;
#pragma unroll
                for (int b = 0; b < K; ++b) xm[g][b] = m[b];
            }
#pragma unroll
            for (int g = 0; g < PG; ++g) {
                const double ax = ncx[B[g]] + nrx[B[g]] * chx;
                const double dy = (ncy[B[g]] + nry[B[g]] * chy) - by;
                const double dy2 = dy * dy;
                double xw[K];
#pragma unroll
                for (int b = 0; b < K; ++b) xw[b] = hw.hw[b] * xm[g][b];
#pragma unroll
                for (int j = 0; j < 4; ++j) hm_entry<K, false, NR>(e4[g][j], ax - bx[j], dy2, xw, c[j]);
            }
        }
    }
    // sum over the 16 columns (lane bits 2..5); row t = 4q' + j is entry j of the
    // lanes with q == q' (lane 4t + (t >> 2) for row t = s)
#pragma unroll
    for (int off = 4; off < kWave; off <<= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < K; ++i) c[j][i] += __shfl_xor(c[j][i], off);
    const int jr = s & 3, srcLane = 4 * s + (s >> 2);
    double* dst = local + ((size_t)n * kRank + s) * K;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double sel = jr == 0 ? c[0][i] : jr == 1 ? c[1][i] : jr == 2 ? c[2][i] : c[3][i];
        const double v = __shfl(sel, srcLane);
        if ((i & 3) == q) dst[i] = hw.om[i] * v;
    }
}


// One entry applied both ways (a canonical pair inside a cluster, k_m2l_hc): the
// forward product o as hm_entry, and the partner's product ob[i] += T_i(c) (E/r) V_A,
// V_A = sum_b T_b(c) xa[b] with xa[b] = (-1)^b hw_b x_A,b(t) (the reversed direction
// has cos = -c; its (-1)^i is applied when ob is flushed).
template <int K, int NR, bool guard0 = false>
__device__ __forceinline__ void hm_entry2(double e, double dx, double dy2, const double (&xw)[K],
                                          const double* __restrict__ xa, double (&o)[K], double (&ob)[K]) {
    const double r2 = __builtin_fma(dx, dx, dy2);
    double ri = rsqrt_nr<NR>(r2);
    if constexpr (guard0) ri = r2 > 0.0 ? ri : 0.0;
    const double c = dx * ri;
    double T[K];
    cheb_T<K>(c, T);
    double v = xw[0], va = xa[0];
#pragma unroll
    for (int b = 1; b < K; ++b) {
        v = __builtin_fma(T[b], xw[b], v);
        va = __builtin_fma(T[b], xa[b], va);
    }
    const double er = e * ri;
    const double av = er * v, ava = er * va;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        o[i] = __builtin_fma(T[i], av, o[i]);
        ob[i] = __builtin_fma(T[i], ava, ob[i]);
    }
}

// the end of a target in the cluster M2L: its 4 x K row sums per lane summed over the
// 16 columns (lane bits 2..5) and added to its LDS locals at `at` (16 x K)
constexpr int kHcMaxWaves = 8;  // the largest cluster workgroup (512 threads)

// The deterministic cluster sums: every add into a cluster's LDS
// slots is an integer add of a fixed-point value (a cluster-wide scale 2^S with the
// slot bound below 2^62, hc_det_scale), so the sums do not depend on the order in which
// the waves add.  fx_of rounds v 2^S to the nearest integer and splits it into the
// two 32-bit words of its two's complement form (|v 2^S| < 2^62: hi fits an int).
__device__ __forceinline__ unsigned long long fx_of(double v, double sc) {
    const double x = __builtin_rint(v * sc);
    const double hi = __builtin_floor(x * 0x1p-32);
    const double lo = __builtin_fma(-hi, 0x1p32, x);  // exact: an integer in [0, 2^32)
    return ((unsigned long long)(unsigned)(int)hi << 32) | (unsigned long long)(unsigned)lo;
}
template <bool DET>
__device__ __forceinline__ void slot_add(double* d, double v, double sc) {
    if constexpr (DET) atomicAdd(reinterpret_cast<unsigned long long*>(d), fx_of(v, sc));
    else atomicAdd(d, v);
}

template <int K, bool DET = false>
__device__ __forceinline__ void m2l_hc_store_target(double (&c)[4][K], double* at, int lane, int s, int q,
                                                    double sc = 0.0) {
    if constexpr (K == 5) {
        // sum over the 16 columns (lane bits 2..5) as a reduce-scatter of the lane's
        // 20 row sums (rows 4q + j, entries i; v = 5 j + i): 20 -> 10 (lane ^ 32),
        // 10 -> 5 (lane ^ 16), 5 -> 3 (lane ^ 8), 3 -> 2 (lane ^ 4); each of the 16
        // column lanes then adds its <= 2 finished sums -- ~90 VALU ops, not ~360
        const bool r4 = xor16_r4(lane);
        const int k32 = swap_add32_f64(1.0, 0.0) > 1.5 ? 0 : 10;  // this lane keeps the first / second half
        const int k16 = swap_add16_f64(1.0, 0.0) > 1.5 ? 0 : 5;
        double v10[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) v10[k] = swap_add32_f64(c[k / 5][k % 5], c[(k + 10) / 5][(k + 10) % 5]);
        double v5[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v5[k] = swap_add16_f64(v10[k], v10[k + 5]);
        const bool h1 = (lane >> 3) & 1, h0 = (lane >> 2) & 1;
        double v3[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // lane ^ 8: h1 = 0 keeps k, h1 = 1 keeps k + 3
            const double x = v5[k], y = k + 3 < 5 ? v5[k + 3] : 0.0;
            v3[k] = (h1 ? y : x) + dpp_f64<0x128>(h1 ? x : y);
        }
        double* d = at;
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // lane ^ 4: h0 = 0 keeps u, h0 = 1 keeps u + 2
            const double x = v3[u], y = u + 2 < 3 ? v3[u + 2] : 0.0;
            const double sum = (h0 ? y : x) + xor16_f64<4>(h0 ? x : y, r4);
            const int w = u + 2 * h0, v2 = w + 3 * h1;
            if (w <= 2 && v2 <= 4) {
                const int v0 = v2 + k16 + k32, j = v0 / 5, i = v0 - 5 * j;
                slot_add<DET>(d + (4 * q + j) * K + i, sum, sc);
            }
        }
    } else {
        {  // sum over the 16 columns (lane bits 2..5) on the VALU: DPP in-row, permlane swaps across rows
            const bool r4 = xor16_r4(lane);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    double v = c[j][i];
                    v += xor16_f64<4>(v, r4);
                    v += xor16_f64<8>(v, r4);
                    v = xsum16_f64(v);
                    c[j][i] = xsum32_f64(v);
                }
        }
        const int jr = s & 3, srcLane = 4 * s + (s >> 2);
        double* d = at + (size_t)s * K;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const double sel = jr == 0 ? c[0][i] : jr == 1 ? c[1][i] : jr == 2 ? c[2][i] : c[3][i];
            const double v = __shfl(sel, srcLane);
            if ((i & 3) == q) slot_add<DET>(d + i, v, sc);
        }
    }
}

// A cluster's LDS slots: its nt targets, then (the halo form) the nh halo nodes whose
// partner products it accumulates for other clusters (Plan::hmHaloPtr).
struct HcSlots {
    int c0, nt, h0, nh;
};

__device__ __forceinline__ HcSlots hc_slots(int cid, const HcArgs& a) {
    HcSlots s;
    s.c0 = a.clPtr[cid];
    s.nt = a.clPtr[cid + 1] - s.c0;
    s.h0 = a.haloPtr ? a.haloPtr[cid] : 0;
    s.nh = a.haloPtr ? a.haloPtr[cid + 1] - s.h0 : 0;
    return s;
}

// the cluster's end: its targets' locals stored, its halo slots stored to their
// partials (both scaled by om; the down pass adds the partials, k_down_tier)
template <int K, bool DET = false>
__device__ __forceinline__ void hc_flush(const HcSlots& c, const HcArgs& a, const double* acc, double isc = 1.0) {
    constexpr int RK = kRank * K;
    auto val = [&](int e) {
        if constexpr (DET) return (double)reinterpret_cast<const long long*>(acc)[e] * isc;
        else return acc[e];
    };
    for (int e = threadIdx.x; e < c.nt * RK; e += blockDim.x) {
        const int k = e / RK, r = e - k * RK;
        a.local[(size_t)a.tgt[c.c0 + k] * RK + r] = a.hw.om[r % K] * val(e);
    }
    const int hb = c.nt * RK;
    for (int e = threadIdx.x; e < c.nh * RK; e += blockDim.x) {
        const int k = e / RK, r = e - k * RK;
        a.hpart[(size_t)a.haloPos[c.h0 + k] * RK + r] = a.hw.om[r % K] * val(hb + e);
    }
}

// DET: the cluster's fixed-point scale.  Every value a slot receives is a sum of
// entries |E T_i (E/r) sum_b T_b hw_b x_b| <= Emax / gap * W(node) (|T| <= 1, E <= Emax,
// r >= the box gap), W(node) = max over its columns of sum_b |hw_b x_b| (k_node_wmax);
// a slot's total is within clBound[c] (the host's 16 columns x the most pairs one
// slot receives x the largest 1/gap of the cluster's pairs, x 2) times Emax times the
// largest W of the nodes the cluster reads.  S puts that bound below 2^62.
__device__ __forceinline__ void hc_det_scale(int cid, const HcSlots& cs, const HcArgs& a, double* red,
                                             double& sc, double& isc) {
    double mw = 0.0;
    for (int k = threadIdx.x; k < cs.nt; k += blockDim.x) mw = fmax(mw, a.wmax[a.tgt[cs.c0 + k]]);
    const int64_t e0 = a.ptr[cs.c0], e1 = a.ptr[cs.c0 + cs.nt];
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) mw = fmax(mw, a.wmax[a.src[e]]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mw = fmax(mw, __shfl_xor(mw, off));
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = mw;
    __syncthreads();
    mw = 0.0;
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) mw = fmax(mw, red[w]);
    const double B = a.clBound[cid] * a.emax[0] * mw;
    int ex = 0;
    if (B > 0.0) (void)frexp(B, &ex);  // B < 2^ex
    const int S = min(1000, max(-1000, 62 - ex));
    sc = ldexp(1.0, S);
    isc = ldexp(1.0, -S);
}

// The same distances for the 4-wave form (LR): from wave-uniform values only,
// dx_j = axs - r cheb_j (one FMA with two scalar operands; ~2-4 % more VALU, but no
// VGPRs held for the target's columns).
__device__ __forceinline__ double cheb_dx_lr(int j, double axs, double r, const Params* __restrict__ P) {
    return __builtin_fma(-r, P->cheb[j], axs);
}

// The harmonic M2L in clusters: one 4-wave workgroup per
// cluster (the active targets of one level under one ancestor kClusterDepth levels
// up), the cluster's locals accumulated in LDS.  Each wave takes the cluster's
// next target from an LDS counter and streams its pair list as k_m2l_hm does; a pair whose
// partner is in the cluster (slot >= 0) is read once, by its smaller id, and also
// yields the partner's product: per lane the 4 rows are summed in registers, the
// quad's lanes by DPP, and the 16 x K result is added to the partner's LDS locals
// (ds_add_f64).  The block stream drops by the in-cluster share (0.65 of the V
// pairs at 64 targets per cluster, tools/vfrac.py); the summation order of the LDS
// adds is not fixed (results repeat to rounding, not bitwise).
// LR: the 4-wave-per-SIMD form (<= 128 VGPRs, k_m2l_hc / k_top_m2l_hc with WPE = 4)
// for launches whose LDS allows 4 workgroups per CU (small clusters: shards)
template <int K, int NR, bool LR = false, bool DET = false>
__device__ __forceinline__ void m2l_hc_cluster(const int cid, const HcArgs& a, double* sm) {
    const int* __restrict__ clPtr = a.clPtr;
    const int* __restrict__ tgt = a.tgt;
    const int64_t* __restrict__ ptr = a.ptr;
    const int* __restrict__ ndir = a.ndir;
    const int* __restrict__ src = a.src;
    const int* __restrict__ blk = a.blk;
    const int* __restrict__ slot = a.slot;
    const double* __restrict__ E = a.E;
    const double* __restrict__ ncx = a.ncx;
    const double* __restrict__ ncy = a.ncy;
    const double* __restrict__ nrx = a.nrx;
    const double* __restrict__ nry = a.nry;
    const Params* __restrict__ P = a.P;
    const HarmWeights& hw = a.hw;
    const double* __restrict__ mult = a.mult;
    constexpr int RK = kRank * K;
    constexpr int PG = 2;
    const HcSlots cs = hc_slots(cid, a);
    const int c0 = cs.c0, nt = cs.nt, nsl = cs.nt + cs.nh;
    (void)clPtr;
    const int nw = (int)(blockDim.x / kWave);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    double* acc = sm;                                     // (nt + nh) x 16 x K: the cluster's locals, its halo
    double* xa = sm + (size_t)nsl * RK + (size_t)w * RK;  // this wave's target multipole, (-1)^b hw_b weighted
    // targets go to the waves dynamically (an LDS counter, in slot order: the low slots
    // own the most in-cluster dual pairs), not round-robin: a wave's load is the sum of
    // its targets' reads, and with 4 targets per wave (shards) the static split left
    // the cluster's slowest wave 5-8 % above the mean
    __shared__ int nextTarget;
    for (int i = threadIdx.x; i < nsl * RK; i += blockDim.x) acc[i] = 0.0;
    if (threadIdx.x == 0) nextTarget = nw;
    [[maybe_unused]] double sc = 0.0, isc = 1.0;
    if constexpr (DET) {
        __shared__ double red[kHcMaxWaves];
        hc_det_scale(cid, cs, a, red, sc, isc);  // (its barrier also publishes the zeroed slots)
    } else {
        __syncthreads();
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int s = lane >> 2, q = lane & 3;
    const double chx = P->cheb[s & 3], chy = P->cheb[s >> 2];
    // the canonical loop's Chebyshev nodes, held in SGPRs: re-loaded per pair they cost
    // a vmcnt(0) that drained every other pair's prefetch (1-2 % of the M2L, r05zk)
    double chu[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) chu[j] = uniform_f64(P->cheb[j]);
    for (int ti = w; ti < nt;) {
        const int n = tgt[c0 + ti];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous target's xa reads are done
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < RK; e += kWave) {
            const int b = e % K;
            xa[e] = ((b & 1) ? -hw.hw[b] : hw.hw[b]) * mult[(size_t)n * RK + e];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // xa visible to every lane of the wave
        __builtin_amdgcn_wave_barrier();
        // the target's Chebyshev x coordinates: held in 8 VGPRs (the 3-wave form; the
        // two-value form cheb_dx measured 3 % slower per block matvec, r03zc), or from
        // wave-uniform values (LR, the 4-wave form, <= 128 VGPRs)
        const double tcx = LR ? ncx[n] : 0.0, trx = nrx[n], tcx1 = ncx[n];
        double bx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[j] = LR ? 0.0 : ncx[n] + trx * P->cheb[j];
        auto dxj = [&](int j, double axs) { return LR ? cheb_dx_lr(j, axs, trx, P) : axs - bx[j]; };
        const double by = ncy[n] + nry[n] * P->cheb[q];
        double c[4][K];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < K; ++i) c[j][i] = 0.0;
        const int64_t p0 = ptr[c0 + ti], pd = p0 + ndir[c0 + ti], p1 = ptr[c0 + ti + 1];
            // directed entries: PG blocks in flight, forward product only; every block
            // is read in its stored orientation (the plan gives a transposed read a
            // directed copy, Plan::hmCopyOwner): two 16-B loads per lane
            for (int64_t cb = p0; cb < pd; cb += kWave) {
                const int cnt = (int)min<int64_t>(kWave, pd - cb);
                const int mySrc = lane < cnt ? src[cb + lane] : 0;
                const int myBlk = lane < cnt ? blk[cb + lane] : 0;
                for (int j0 = 0; j0 < cnt; j0 += PG) {
                    double e4[PG][4];
                    double xm[PG][K];
                    int B[PG];
    #pragma unroll
                    for (int g = 0; g < PG; ++g) {
                        const int b = __builtin_amdgcn_readlane(myBlk, min(j0 + g, cnt - 1));
                        const dbl2* p = reinterpret_cast<const dbl2*>(E + (size_t)b * 256 + 16 * s + 4 * q);
                        const dbl2 k0 = p[0], k1 = p[1];
                        const bool ok = j0 + g < cnt;  // a skipped slot re-reads a valid block
                        e4[g][0] = ok ? k0.x : 0.0;
                        e4[g][1] = ok ? k0.y : 0.0;
                        e4[g][2] = ok ? k1.x : 0.0;
                        e4[g][3] = ok ? k1.y : 0.0;
                    }
    #pragma unroll
                    for (int g = 0; g < PG; ++g) {  // a skipped block's source is a valid clamp; its E is zero
                        B[g] = __builtin_amdgcn_readlane(mySrc, min(j0 + g, cnt - 1));
                        const double* m = mult + ((size_t)B[g] * kRank + s) * K;
    #pragma unroll
                        for (int b = 0; b < K; ++b) xm[g][b] = m[b];
                    }
    #pragma unroll
                    for (int g = 0; g < PG; ++g) {
                        const double axs = LR ? (ncx[B[g]] - tcx) + nrx[B[g]] * chx : ncx[B[g]] + nrx[B[g]] * chx;
                        const double dy = (ncy[B[g]] + nry[B[g]] * chy) - by;
                        const double dy2 = dy * dy;
                        double xw[K];
    #pragma unroll
                        for (int b = 0; b < K; ++b) xw[b] = hw.hw[b] * xm[g][b];
    #pragma unroll
                        for (int j = 0; j < 4; ++j) hm_entry<K, false, NR>(e4[g][j], dxj(j, axs), dy2, xw, c[j]);
                    }
                }
            }
            // canonical entries (stored as read): both products, the partner's into its
            // LDS slot (a cluster target, or a halo slot in the halo form); the next
            // pair's block, source multipole and box are loaded before this pair's
            // arithmetic (two blocks in flight per wave: in the halo form every pair is
            // here)
            for (int64_t cb = pd; cb < p1; cb += kWave) {
                const int cnt = (int)min<int64_t>(kWave, p1 - cb);
                const int mySrc = lane < cnt ? src[cb + lane] : 0;
                const int myBlk = lane < cnt ? blk[cb + lane] : 0;
                // LR: the partner's slot by a scalar load (needed only at the flush), one
                // VGPR fewer across the stream
                const int mySlot = !LR && lane < cnt ? slot[cb + lane] : 0;
                dbl2 k0, k1;
                double xm[K], gcx, grx, gcy, gry;
                auto fetch = [&](int jj, dbl2& a0, dbl2& a1, double (&x)[K], double& fcx, double& frx, double& fcy,
                                 double& fry) {
                    const int b = __builtin_amdgcn_readlane(myBlk, jj);
                    const int B = __builtin_amdgcn_readlane(mySrc, jj);
                    const dbl2* p = reinterpret_cast<const dbl2*>(E + (size_t)b * 256 + 16 * s + 4 * q);
                    a0 = p[0];
                    a1 = p[1];
                    const double* m = mult + ((size_t)B * kRank + s) * K;
    #pragma unroll
                    for (int bb = 0; bb < K; ++bb) x[bb] = m[bb];
                    fcx = ncx[B];
                    frx = nrx[B];
                    fcy = ncy[B];
                    fry = nry[B];
                };
                // pair jj from one register set while the next pair loads into the
                // other (unrolled by two: no register copies between the sets)
                auto pair = [&](int jj, const dbl2& a0, const dbl2& a1, const double (&xv)[K], double fcx,
                                double frx, double fcy, double fry) {
                    const int sl = LR ? slot[cb + jj] : __builtin_amdgcn_readlane(mySlot, jj);
                    // the distances from wave-uniform values (as the LR form): 8 VGPRs
                    // fewer than the held target columns bx, the same VALU count
                    const double axs = (fcx - tcx1) + frx * chx;
                    const double dy = (fcy + fry * chy) - by;
                    const double dy2 = dy * dy;
                    double xw[K], ob[K];
    #pragma unroll
                    for (int bb = 0; bb < K; ++bb) {
                        xw[bb] = hw.hw[bb] * xv[bb];
                        ob[bb] = 0.0;
                    }
                    const double e4[4] = {a0.x, a0.y, a1.x, a1.y};
    #pragma unroll
                    for (int j = 0; j < 4; ++j)
                        hm_entry2<K, NR>(e4[j], __builtin_fma(-trx, chu[j], axs), dy2, xw, xa + (4 * q + j) * K, c[j], ob);
    #pragma unroll
                    for (int i = 0; i < K; ++i) ob[i] = quad_sum(ob[i]);  // rows 4q'+j over the quad
                    double* d = acc + ((size_t)sl * kRank + s) * K;
                    if constexpr (DET) {
                        // the quad's lanes share the K conversions: lane q adds entries q, q + 4, ..
                        const double sq = (q & 1) ? -sc : sc;
    #pragma unroll
                        for (int i0 = 0; i0 < K; i0 += 4) {
                            double v = ob[i0];
    #pragma unroll
                            for (int u = 1; u < 4; ++u)
                                if (i0 + u < K && q == u) v = ob[i0 + u];
                            if (i0 + q < K) slot_add<true>(d + i0 + q, v, sq);
                        }
                    } else if (q == 0) {
    #pragma unroll
                        for (int i = 0; i < K; ++i) atomicAdd(d + i, (i & 1) ? -ob[i] : ob[i]);
                    }
                };
                dbl2 m0, m1;
                double xn[K], hcx, hrx, hcy, hry;
                fetch(0, k0, k1, xm, gcx, grx, gcy, gry);
                for (int jj = 0; jj < cnt; jj += 2) {
                    // the next pair (the last one again at the end: an L1 hit, no branch
                    // for the wait counts to merge over)
                    fetch(min(jj + 1, cnt - 1), m0, m1, xn, hcx, hrx, hcy, hry);
                    pair(jj, k0, k1, xm, gcx, grx, gcy, gry);
                    if (jj + 1 >= cnt) break;
                    fetch(min(jj + 2, cnt - 1), k0, k1, xm, gcx, grx, gcy, gry);
                    pair(jj + 1, m0, m1, xn, hcx, hrx, hcy, hry);
                }
            }
        m2l_hc_store_target<K, DET>(c, acc + (size_t)ti * kRank * K, lane, s, q, sc);
        int nx = 0;
        if (lane == 0) nx = atomicAdd(&nextTarget, 1);
        ti = __builtin_amdgcn_readlane(nx, 0);
    }
    __syncthreads();
    hc_flush<K, DET>(cs, a, acc, isc);
}

// ---- the ring form of the cluster M2L ----
//
// m2l_hc_cluster keeps one block (two in the directed loop) in flight per wave:
// every pair is a dependent HBM round trip (~1.7 us per block per wave at 1 and at 8
// shards, tools/top_trace.py), and deeper register prefetch does not fit beside the
// 40 accumulator VGPRs at 3 waves per SIMD.  Here each wave streams its pair list
// through a private ring of D slots in LDS filled by LDS-DMA (global_load_lds_dwordx4:
// no VGPR holds a block in flight): slot = the 2 KB E block, the source's 16 x K
// multipole and its box (cx, cy, rx, ry).  The wave issues pair k + D - 1, waits with
// a counted vmcnt for pair k and computes it from LDS, so D - 1 blocks stay in flight
// across the compute.  The target's own weighted multipole (the dual products'
// operand) lives in registers.
//
// The compiler's wait-count pass treats every LDS access as possibly reading an
// LDS-DMA destination and would put vmcnt(0) before it, draining the ring.  So every
// LDS access inside the stream is inline asm, which that pass does not see: the slot
// reads (closed by one lgkmcnt(0) that re-defines their outputs) and the partner
// products' ds_add_f64; the counted vmcnt waits are asm too.
constexpr int kRingMaxK = 5;  // the ring forms compile without spills up to 5 blocks (hm_ring_xl)

template <int K>
struct Ring {
    static_assert(K <= kRingMaxK, "the ring form spills above 5 blocks");
    static constexpr int kMultB = kRank * K * 8;        // the multipole's bytes
    static constexpr int kMultL = kMultB / 16;          // its 16-byte lanes
    static constexpr bool kSplit = kMultL + 2 > kWave;  // the box in an instruction of its own (K = 8)
    static constexpr int kNI = kSplit ? 4 : 3;          // LDS-DMA instructions per slot
    static constexpr int kSlot = 2048 + kMultB + 32;    // bytes per slot
};

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ unsigned lds_offset(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ void glds16(const double* g, unsigned lds) {
    __builtin_amdgcn_global_load_lds(g, (lds_void*)(uintptr_t)lds, 16, 0, 0);
}

// no "memory" clobbers on the stream's asm: one would make every later global load of
// the kernel a vector load (the wave-uniform pair indices must stay scalar loads, or
// their vmcnt waits drain the ring); volatile asm keeps its order with the LDS-DMA
// intrinsics and with each other
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N));
}

// wait until the slot issued `after` slots ago (0 .. 3) has landed
template <int NI>
__device__ __forceinline__ void ring_wait(int after) {
    if (after >= 3) wait_vm<3 * NI>();
    else if (after == 2) wait_vm<2 * NI>();
    else if (after == 1) wait_vm<NI>();
    else wait_vm<0>();
}

// fill a slot: block b of E, multipole and box of source node B (wave-uniform b, B)
template <int K>
__device__ __forceinline__ void ring_issue(const double* __restrict__ E, const double* __restrict__ mult,
                                           const double* __restrict__ geo, int b, int B, unsigned slot, int lane) {
    using R = Ring<K>;
    const double* eg = E + (size_t)b * 256 + 2 * lane;
    glds16(eg, slot);
    glds16(eg + 128, slot + 1024);
    const double* mg = mult + (size_t)B * (kRank * K) + 2 * lane;
    const double* gg = geo + 4 * (size_t)B + 2 * (lane - (R::kSplit ? 0 : R::kMultL));
    if constexpr (R::kSplit) {
        glds16(mg, slot + 2048);
        if (lane < 2) glds16(gg, slot + 2048 + R::kMultB);
    } else {
        if (lane < R::kMultL + 2) glds16(lane < R::kMultL ? mg : gg, slot + 2048);
    }
}

// lane (s, q)'s operands from a landed slot: rows 4q .. 4q+3 of column s of the
// block, the source multipole's row s, the source box
template <int K>
__device__ __forceinline__ void ring_read(unsigned slot, int lane, int s, double (&e4)[4], double (&xm)[K],
                                          double (&g)[4]) {
    using R = Ring<K>;
    const unsigned eo = slot + 32 * lane, go = slot + 2048 + R::kMultB, mo = slot + 2048 + 8 * K * s;
    dbl2 e01, e23, g01, g23;
    asm volatile("ds_read_b128 %0, %1" : "=v"(e01) : "v"(eo));
    asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(e23) : "v"(eo));
    asm volatile("ds_read_b128 %0, %1" : "=v"(g01) : "v"(go));
    asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(g23) : "v"(go));
#pragma unroll
    for (int b = 0; b < K; ++b) asm volatile("ds_read_b64 %0, %1" : "=v"(xm[b]) : "v"(mo + 8 * b));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(e01), "+v"(e23), "+v"(g01), "+v"(g23));
#pragma unroll
    for (int b = 0; b < K; ++b) asm volatile("" : "+v"(xm[b]));
    e4[0] = e01.x;
    e4[1] = e01.y;
    e4[2] = e23.x;
    e4[3] = e23.y;
    g[0] = g01.x;
    g[1] = g01.y;
    g[2] = g23.x;
    g[3] = g23.y;
}

// rows 4q .. 4q+3 of the wave's weighted target multipole (4K doubles from `off`)
template <int K>
__device__ __forceinline__ void ring_read_xa(unsigned off, double (&x)[4 * K]) {
    dbl2 v[2 * K];
#pragma unroll
    for (int i = 0; i < 2 * K; ++i) asm volatile("ds_read_b128 %0, %1" : "=v"(v[i]) : "v"(off + 16 * i));
    asm volatile("s_waitcnt lgkmcnt(0)");
#pragma unroll
    for (int i = 0; i < 2 * K; ++i) {
        asm volatile("" : "+v"(v[i]));
        x[2 * i] = v[i].x;
        x[2 * i + 1] = v[i].y;
    }
}

template <int K, int NR, int D, bool XL>
__device__ __forceinline__ void m2l_hcr_cluster(const int cid, const HcArgs& a, double* sm) {
    static_assert(D >= 2 && D <= 4, "ring depth");
    using R = Ring<K>;
    const int* __restrict__ clPtr = a.clPtr;
    const int* __restrict__ tgt = a.tgt;
    const int64_t* __restrict__ ptr = a.ptr;
    const int* __restrict__ ndir = a.ndir;
    const int* __restrict__ src = a.src;
    const int* __restrict__ blk = a.blk;
    const int* __restrict__ slot = a.slot;
    const double* __restrict__ E = a.E;
    const double* __restrict__ geo = a.geo;
    const double* __restrict__ ncx = a.ncx;
    const double* __restrict__ ncy = a.ncy;
    const double* __restrict__ nrx = a.nrx;
    const double* __restrict__ nry = a.nry;
    const Params* __restrict__ P = a.P;
    const HarmWeights& hw = a.hw;
    const double* __restrict__ mult = a.mult;
    constexpr int RK = kRank * K;
    const HcSlots cs = hc_slots(cid, a);
    const int c0 = cs.c0, nt = cs.nt, nsl = cs.nt + cs.nh;
    (void)clPtr;
    const int nw = (int)(blockDim.x / kWave);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    double* acc = sm;                                                       // (nt + nh) x 16 x K: locals, halo
    double* xl = sm + (size_t)nsl * RK + (XL ? (size_t)w * RK : 0);         // XL: this wave's target multipole
    const unsigned ring = lds_offset(sm + (size_t)nsl * RK + (XL ? (size_t)nw * RK : 0)) + (unsigned)(w * D * R::kSlot);
    const unsigned accOff = lds_offset(acc);
    for (int i = threadIdx.x; i < nsl * RK; i += blockDim.x) acc[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const int s = lane >> 2, q = lane & 3;
    const double chx = P->cheb[s & 3], chy = P->cheb[s >> 2];
    for (int ti = w; ti < nt; ti += nw) {
        const int n = tgt[c0 + ti];
        // the target's multipole rows 4q + j, (-1)^b hw_b weighted (the dual products):
        // in registers (40 VGPRs at K = 5, 2 waves per SIMD), or (XL) in LDS, read per
        // dual block (3 waves per SIMD)
        double xa[XL ? 1 : 4][K];
        if constexpr (XL) {
            for (int e = lane; e < RK; e += kWave) {
                const int b = e % K;
                xl[e] = ((b & 1) ? -hw.hw[b] : hw.hw[b]) * mult[(size_t)n * RK + e];
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // xl visible to every lane of the wave
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int b = 0; b < K; ++b)
                    xa[j][b] = ((b & 1) ? -hw.hw[b] : hw.hw[b]) * mult[(size_t)n * RK + (4 * q + j) * K + b];
        }
        double bx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bx[j] = ncx[n] + nrx[n] * P->cheb[j];
        const double by = ncy[n] + nry[n] * P->cheb[q];
        double c[4][K];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < K; ++i) c[j][i] = 0.0;
        const int64_t p0 = ptr[c0 + ti], pd = p0 + ndir[c0 + ti], p1 = ptr[c0 + ti + 1];
        // the pair list in chunks of 64: its indices in lanes (one vector load each, while
        // the ring is empty -- the compiler's wait for them would drain it), the ring
        // filled and drained per chunk
        for (int64_t cb = p0; cb < p1; cb += kWave) {
            const int cnt = (int)min<int64_t>(kWave, p1 - cb);
            const int mySrc = lane < cnt ? src[cb + lane] : 0;
            const int myBlk = lane < cnt ? blk[cb + lane] : 0;
            const int mySlot = lane < cnt && cb + lane >= pd ? slot[cb + lane] : 0;
            const int nDir = (int)max<int64_t>(0, min<int64_t>(cnt, pd - cb));  // directed entries of the chunk
            for (int k = 0; k < D - 1 && k < cnt; ++k)
                ring_issue<K>(E, mult, geo, __builtin_amdgcn_readlane(myBlk, k), __builtin_amdgcn_readlane(mySrc, k),
                              ring + k * R::kSlot, lane);
            int cur = 0;  // the slot of pair k
            for (int k = 0; k < cnt; ++k) {
                int after = cnt - 1 - k;
                if (k + D - 1 < cnt) {
                    const int ns = cur == 0 ? D - 1 : cur - 1;  // the slot pair k - 1 used: free again
                    ring_issue<K>(E, mult, geo, __builtin_amdgcn_readlane(myBlk, k + D - 1),
                                  __builtin_amdgcn_readlane(mySrc, k + D - 1), ring + ns * R::kSlot, lane);
                    after = D - 1;
                }
                ring_wait<R::kNI>(after);
                double e4[4], xm[K], g[4];
                ring_read<K>(ring + cur * R::kSlot, lane, s, e4, xm, g);
                cur = cur == D - 1 ? 0 : cur + 1;
                const double ax = g[0] + g[2] * chx;
                const double dy = (g[1] + g[3] * chy) - by;
                const double dy2 = dy * dy;
                double xw[K];
#pragma unroll
                for (int b = 0; b < K; ++b) xw[b] = hw.hw[b] * xm[b];
                if (k < nDir) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) hm_entry<K, false, NR>(e4[j], ax - bx[j], dy2, xw, c[j]);
                } else {
                    double ob[K];
#pragma unroll
                    for (int b = 0; b < K; ++b) ob[b] = 0.0;
                    if constexpr (XL) {
                        double xr[4 * K];
                        ring_read_xa<K>(lds_offset(xl) + 32 * K * q, xr);
#pragma unroll
                        for (int j = 0; j < 4; ++j) hm_entry2<K, NR>(e4[j], ax - bx[j], dy2, xw, xr + j * K, c[j], ob);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) hm_entry2<K, NR>(e4[j], ax - bx[j], dy2, xw, xa[j], c[j], ob);
                    }
#pragma unroll
                    for (int i = 0; i < K; ++i) ob[i] = quad_sum(ob[i]);  // rows 4q'+j over the quad
                    if (q == 0) {
                        const int sl = __builtin_amdgcn_readlane(mySlot, k);
                        const unsigned d = accOff + (unsigned)(((sl * kRank + s) * K) * 8);
#pragma unroll
                        for (int i = 0; i < K; ++i)
                            asm volatile("ds_add_f64 %0, %1" ::"v"(d + 8 * i), "v"((i & 1) ? -ob[i] : ob[i]));
                    }
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)");  // the partner adds, before the compiler's LDS ops
        m2l_hc_store_target<K>(c, acc + (size_t)ti * RK, lane, s, q);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    hc_flush<K>(cs, a, acc);
}

template <int K, int NR, int D, bool XL, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) k_m2l_hcr(HcArgs a) {
    extern __shared__ double sm[];
    m2l_hcr_cluster<K, NR, D, XL>((int)blockIdx.x, a, sm);
}

// WPE, the cluster form's occupancy: 3 = 4-wave workgroups at 3 waves per SIMD (3 per
// CU); 6 = 6-wave workgroups at 3 waves per SIMD (2 per CU: the halo form's 64-target
// clusters need ~72 KB of LDS); 4 = the LR form (<= 128 VGPRs) in 4-wave workgroups;
// 8 = the LR form with 8 waves (512 threads) per cluster, 2 clusters per CU
template <int WPE>
constexpr int kHcThreads = WPE == 8 ? 512 : WPE == 6 ? 384 : 256;
template <int WPE>
constexpr int kHcWaves = WPE == 8 ? 4 : WPE == 6 ? 3 : WPE;
template <int WPE>
constexpr bool kHcLR = WPE == 4 || WPE == 8;

template <int K, int NR, int WPE, bool DET = false>
__global__ void __launch_bounds__(kHcThreads<WPE>) __attribute__((amdgpu_waves_per_eu(kHcWaves<WPE>)))
k_m2l_hc(HcArgs a) {
    extern __shared__ double sm[];
    m2l_hc_cluster<K, NR, kHcLR<WPE>, DET>((int)blockIdx.x, a, sm);
}

// ----------------------------------------------------------------- fused top of tree + M2L
//
// The upper up tiers are a few hundred small, latency-bound tasks; as launches of
// their own they sit between the bottom tier and the M2L on every apply (and on every
// rank of a sharded one, where they do not shrink with the rank count).  Here they
// run as the first blocks of the M2L launch: the clusters that need none of their
// multipoles (the finest levels: all but a few percent of the work) stream from the
// start, and the rest wait for the tier they read (TopArgs.clWait, Plan::hmClWait).
// Hand-off per tier: a counter of finished tasks, published after an agent-scope
// release by each task and polled (relaxed, agent scope) by one lane of a waiting
// block, which then acquires before its block reads (MI355X_MICROARCH.md, cross-
// workgroup visibility).
// No dispatch-order assumption: a wait that has polled spinLimit times without
// seeing the tier complete computes the tier's tasks itself (top_ensure), after the
// tiers below it, the same way.  up_task only assigns (mult, the gathered roots), so
// a task computed twice -- by its own block and by a waiter -- writes the same bits,
// and a waiter reads only what it computed itself or what a completed counter
// published.  So the launch cannot hang on, or be spoiled by, a producer block that
// is not resident; each such computation counts in TopArgs.steals (aniso_stats).
typedef __attribute__((address_space(1))) unsigned gu32;

// one lane polls tier k's counter up to spinLimit times; true (and acquired) if the tier completed
__device__ __forceinline__ bool top_poll(const TopArgs& t, int k, unsigned target) {
    __shared__ int done;
    if (threadIdx.x == 0) {
        gu32* c = (gu32*)(t.cnt + k);
        bool ok = false;
        for (unsigned spins = 0;; ++spins) {
            if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
                ok = true;
                break;
            }
            if (spins >= t.spinLimit) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        done = ok ? 1 : 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool ok = done != 0;
    __syncthreads();  // `done` is reused by the next poll
    return ok;
}

// tiers 1 .. k complete for this block: the highest tier whose counter completes within
// the poll bound, then every task of the tiers above it computed here, bottom up
template <int K>
__device__ __forceinline__ void top_ensure(const TopArgs& t, const UpArgs& u, int k, double* sm) {
    int j = k;
    while (j >= 1 && !top_poll(t, j, (unsigned)(t.blk0[j + 1] - t.blk0[j]))) --j;
    for (int jj = j + 1; jj <= k; ++jj) {
        const int nj = t.blk0[jj + 1] - t.blk0[jj];
        for (int i = 0; i < nj; ++i) {
            up_task<K>(t.task0[jj] + i, u.maxTask, u.desc, u.grpFix, u.node, u.code, u.geom, u.leafRange, u.pxT,
                       u.pyT, u.xin, u.ldi, u.treeIn, u.perm, u.sigT, u.wT, u.fT, u.cT, u.P, u.mult, u.rootSlot,
                       jj == 1 ? t.recv1 : nullptr, nullptr, nullptr, sm);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // its mult stores, read by the next task
            __syncthreads();
        }
        if (threadIdx.x == 0 && t.steals)
            __hip_atomic_fetch_add((gu32*)t.steals, (unsigned)nj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ void top_publish(unsigned* cnt, int k) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep: the fence's own wait can be dropped
        __hip_atomic_fetch_add((gu32*)(cnt + k), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// development timeline of the fused launch (ANISO_TOP_TRACE=1, tools/top_trace.py):
// per block the 100 MHz wall clock at its start, after its wait and at its end, and
// the hardware slot it ran on (HW_ID: wave / SIMD / CU / SE bits; XCC_ID above)
template <bool TRACE>
__device__ __forceinline__ void top_mark(const TopArgs& t, int field) {
    if constexpr (!TRACE) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t* r = t.trace + 4 * (int64_t)blockIdx.x;
        r[field] = (int64_t)__builtin_amdgcn_s_memrealtime();
        if (field == 0)
            r[3] = (int64_t)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) |
                   ((int64_t)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) << 32);
    }
}

template <int K, int NR, int D, bool XL, bool LR = false>
__device__ __forceinline__ void m2l_cluster_form(int cid, const HcArgs& a, double* sm) {
    if constexpr (D == 0) m2l_hc_cluster<K, NR, LR>(cid, a, sm);
    else m2l_hcr_cluster<K, NR, D, XL>(cid, a, sm);
}

template <int K, int U, int NR, bool FUSE, bool SYM = false, bool UP = false>
__device__ __forceinline__ void near_hs_group(int g, const NearHsArgs& n, double* tab);

// NEAR: the staged near field's groups (k_near_hs with fused corrections) are the last
// blocks (ANISO_NEAR_IN_TOP).  The dispatcher hands out blocks in
// order, so they take the slots the clusters free at the launch's tail.
template <int K, int NR, int WPE, int D, bool XL, bool TRACE = false, bool NEAR = false>
__global__ void __launch_bounds__(kHcThreads<WPE>) __attribute__((amdgpu_waves_per_eu(kHcWaves<WPE>)))
k_top_m2l_hc(UpArgs u, TopArgs t, HcArgs a, NearHsArgs n) {
    extern __shared__ double sm[];
    const int b = (int)blockIdx.x;
    top_mark<TRACE>(t, 0);
    if (b < t.nUp) {
        int k = 1;
        while (b >= t.blk0[k + 1]) ++k;
        if (k >= 2) top_ensure<K>(t, u, k - 1, sm);
        top_mark<TRACE>(t, 1);
        up_task<K>(t.task0[k] + (b - t.blk0[k]), u.maxTask, u.desc, u.grpFix, u.node, u.code, u.geom, u.leafRange,
                   u.pxT, u.pyT, u.xin, u.ldi, u.treeIn, u.perm, u.sigT, u.wT, u.fT, u.cT, u.P, u.mult, u.rootSlot,
                   k == 1 ? t.recv1 : nullptr, nullptr, nullptr, sm);
        top_publish(t.cnt, k);
        top_mark<TRACE>(t, 2);
        return;
    }
    const int cid = b - t.nUp;
    if constexpr (NEAR) {
        if (cid >= t.nCl) {
            top_mark<TRACE>(t, 1);
            near_hs_group<K, 4, 2, true>(cid - t.nCl, n, sm);
            top_mark<TRACE>(t, 2);
            return;
        }
    }
    const int w = t.clWait[cid];
    if (w > 0) {  // its own copy: behind the wait's fence the source boxes load through the vector path
        top_ensure<K>(t, u, w, sm);
        top_mark<TRACE>(t, 1);
        m2l_cluster_form<K, NR, D, XL, kHcLR<WPE>>(cid, a, sm);
        top_mark<TRACE>(t, 2);
        return;
    }
    // no store or fence on the way here, so the compiler keeps the wave-uniform
    // source-box reads (ncx[B] ...) on scalar loads as in k_m2l_hc
    top_mark<TRACE>(t, 1);
    m2l_cluster_form<K, NR, D, XL, kHcLR<WPE>>(cid, a, sm);
    top_mark<TRACE>(t, 2);
}

// ----------------------------------------------------------------- near field

// U/W near field (bbfmm.h:1081-1099) for every mode of the block matvec, directed
// E blocks (column-major nT4 x S per target leaf, rows padded to a multiple of 4,
// the layout of k_cache_near): G lanes per target leaf (G = 16: leaves <= 16 points,
// 4 leaves per wave; else 64), lane (row quad rq, column phase) computes rows
// 4rq..4rq+3 for its columns, U columns in flight; the sources' points and charges
// are read straight from pxT / pyT / fT (the lanes of a column share the lines).
// out (stored, not added) = scale * (sum over sources + the mode-0 diagonal).
template <int K, int G, int U, int NR, bool XCD = false>
__global__ void __launch_bounds__(256) k_near_hm(int nl, const int4* __restrict__ leafInfo,
                                                 const int64_t* __restrict__ nearPtsPtr,
                                                 const int* __restrict__ nearPts, const int64_t* __restrict__ nearKOff,
                                                 const double* __restrict__ E, const double* __restrict__ pxT,
                                                 const double* __restrict__ pyT, const double* __restrict__ sigDiag,
                                                 HarmWeights hw, const double* __restrict__ fT,
                                                 const int* __restrict__ operm, int64_t obase, int64_t ldo,
                                                 int flags, double scale, double* __restrict__ out) {
    static_assert(G == 16 || G == 64, "leaf group of 16 or 64 lanes");
    constexpr int KS = kStride<K>;
    const int gl = threadIdx.x & (G - 1);
    const int bid = XCD ? xcd_tile((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;  // XCD: contiguous leaves per L2
    const int li = (int)(((int64_t)bid * blockDim.x + threadIdx.x) / G);
    const bool active = li < nl;
    int4 info = make_int4(0, 0, 0, 0);
    int64_t pb = 0, koff = 0;
    if (active) {
        info = leafInfo[li];
        pb = nearPtsPtr[li];
        koff = nearKOff[li];
    }
    const bool nearOn = (flags & kStageNear) != 0;
    const int nT = info.z, S = nearOn ? info.w : 0;
    const int64_t tb = info.y;
    const int nq = (nT + 3) >> 2;  // row quads
    const int cstr = 2 * nq;       // column stride in 16-B units
    int lpc = 4;                   // lanes per column (G = 16: leaves <= 16 points, 4 quads)
    if constexpr (G == 64) {
        lpc = 1;
        while (lpc < nq && lpc < kWave) lpc <<= 1;
    }
    const int cps = G / lpc, cph = gl / lpc;
    for (int rc = 0; rc < nq || rc == 0; rc += G) {  // > 64 row quads: leaves over 256 points
        const int rq = rc + (gl & (lpc - 1));
        const bool rowOk = active && rq < nq;
        double tx[4], ty[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = min(4 * rq + j, max(nT - 1, 0));  // padded rows: E is zero there
            tx[j] = rowOk ? pxT[tb + t] : 0.0;
            ty[j] = rowOk ? pyT[tb + t] : 0.0;
        }
        double a[4][K];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < K; ++i) a[j][i] = 0.0;
        if (rowOk) {
            const dbl2* kc = reinterpret_cast<const dbl2*>(E + koff) + 2 * rq;
            for (int c0 = cph; c0 < S; c0 += U * cps) {
                int ix[U];
#pragma unroll
                for (int u = 0; u < U; ++u) ix[u] = nearPts[pb + min(c0 + u * cps, S - 1)];
                dbl2 kk[U][2];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int sc = c0 + u * cps;
                    const dbl2* p = kc + (size_t)min(sc, S - 1) * cstr;
                    const bool ok = sc < S;
                    kk[u][0] = ok ? __builtin_nontemporal_load(p) : dbl2{0.0, 0.0};
                    kk[u][1] = ok ? __builtin_nontemporal_load(p + 1) : dbl2{0.0, 0.0};
                }
                double f[U][K], sx[U], sy[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    load_charges<K>(fT + (size_t)ix[u] * KS, f[u]);
                    sx[u] = pxT[ix[u]];
                    sy[u] = pyT[ix[u]];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    double xw[K];
#pragma unroll
                    for (int b = 0; b < K; ++b) xw[b] = hw.hw[b] * f[u][b];
                    const double e4[4] = {kk[u][0].x, kk[u][0].y, kk[u][1].x, kk[u][1].y};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const double dy = sy[u] - ty[j];
                        hm_entry<K, true, NR>(e4[j], sx[u] - tx[j], dy * dy, xw, a[j]);
                    }
                }
            }
        }
        // sum over the column phases
        if constexpr (G == 16) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    double v = a[j][i];
                    v += dpp_f64<0x124>(v);  // row_ror:4
                    v += dpp_f64<0x128>(v);  // row_ror:8
                    a[j][i] = v;
                }
        } else {
            for (int off = lpc; off < kWave; off <<= 1)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < K; ++i) a[j][i] += __shfl_xor(a[j][i], off);
        }
        if (rowOk) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = 4 * rq + j;
                const bool mine = (G == 16) ? (cph == j) : (cph == 0);
                if (!mine || t >= nT) continue;
                const int64_t k = tb + t;
                double f[K];
                load_charges<K>(fT + (size_t)k * KS, f);
                const double sd = nearOn ? sigDiag[k] : 0.0;
                const int64_t oi = out_index(operm, obase, k);
#pragma unroll
                for (int i = 0; i < K; ++i)
                    out[(size_t)i * ldo + oi] = hw.om[i] * scale * __builtin_fma(hw.dw[i] * sd, f[i], a[j][i]);
            }
        }
        if constexpr (G == 16) break;
    }
}

// The same near field (leaves <= 16 points) with the sources staged in LDS: one
// workgroup = 16 consecutive leaves (a 4 x 4 leaf block on a uniform grid) whose
// U/W source points form one table (Plan::nsPts: their union, ~36 leaves instead
// of 16 x 9 per-column gathers); the table rows (x, y, charges) are loaded once,
// coalesced, and every column then reads its source from LDS by its 16-bit row
// (nearLoc).  Only the E stream stays in HBM.  Same lane layout as k_near_hm<G=16>.

// Table row stride: x, y, the K charges, rounded up to an odd number of doubles, so the
// up to 16 different rows one wave reads at a time fall on different LDS banks (an
// even stride of 8 doubles put every 4th row on the same banks).  K = 5: 7 doubles
// (not 9), so a 16-leaf group's table takes 32 KB instead of 41 KB at 1M points.
template <int K>
constexpr int kTabRow = (K + 2) | 1;

// The bottom up tier in the staged near field (NearHsArgs::upMult): group g's 16
// leaves are one tier-0 subtree, leaf slots 4m .. 4m + 3 under parent m
// (Plan::nearUpGrp).  Out of the group's table region once the epilogue is done with it:
//  * each lane stores its point's Chebyshev weights and weighted charges (the
//    epilogue's point t = 4 (ln & 3) + (ln >> 2) of leaf slot l; zero past the leaf);
//  * P2M (bbfmm.h:737-748): lane ln of leaf l sums entry ln = (i, j) of the leaf's
//    multipole over the leaf's 16 points, every right-hand side, in point order;
//  * M2M (bbfmm.h:855-859) to the parents: one lane per (parent, row, child), the 4
//    children's partial rows of a parent added by a DPP quad reduction (fixed order,
//    as up_task's), then the root the same way from the parents.
// Transfer matrices from global memory (8 KB, cache-resident).
template <int K>
__device__ __forceinline__ void near_up_tail(int g, bool active, int nT, int64_t tb, int leafNode,
                                             const NearHsArgs& n, double (&f)[K], double* tab) {
    constexpr int RK = kRank * K;
    constexpr int PW = 2 * kNP + K;  // per point: Sx, Sy, f
    const int ln = threadIdx.x & 15, l = (int)(threadIdx.x >> 4);
    const int t = 4 * (ln & 3) + (ln >> 2);
    const bool on = active && t < nT;
    const int64_t kp = tb + (on ? t : 0);
    const int* G = n.upGrp + (size_t)g * kNearUpInts;
    const Params* __restrict__ P = n.upP;
    // the tail's global reads issued ahead of the stage that uses them (the near loop's
    // registers are free now): the M2M row of this lane's child quadrant (G[4 m + c] & 3)
    // here, before the first barrier; the root's row (parent slot m: G[16 + m] = m,
    // Plan::buildNearUp) at the start of the M2M stage
    const int um = threadIdx.x >> 6, ur = (threadIdx.x >> 2) & 15, uc = threadIdx.x & 3;
    const int code = G[4 * um + uc];
    const int parentNode = G[20 + um], rootNode = G[24];
    double Rc[kRank];
    {
        const double* R = &P->R[code & 3][ur * kRank];
#pragma unroll
        for (int rr = 0; rr < kRank; ++rr) Rc[rr] = R[rr];
    }
    double Sx[kNP], Sy[kNP];
    {
        const int nd = active ? leafNode : 0;
        const double cx = n.upNcx[nd], cy = n.upNcy[nd], irx = 1.0 / n.upNrx[nd], iry = 1.0 / n.upNry[nd];
        cheb_weights(P, (n.pxT[kp] - cx) * irx, Sx);
        cheb_weights(P, (n.pyT[kp] - cy) * iry, Sy);
    }
    double* PT = tab;              // 256 points x PW; leaf l's rows reused for its multipole (16 x K <= 16 PW)
    double* PM = tab + 256 * PW;   // the 4 parents, 16 x K each
    __syncthreads();  // every lane is done with the source table (the epilogue's corrections read it)
    {
        double* q = PT + (size_t)threadIdx.x * PW;
#pragma unroll
        for (int i = 0; i < kNP; ++i) {
            q[i] = Sx[i];
            q[kNP + i] = Sy[i];
        }
#pragma unroll
        for (int b = 0; b < K; ++b) q[2 * kNP + b] = on ? f[b] : 0.0;
    }
    __syncthreads();
    {
        const int i = ln & 3, j = ln >> 2;
        const double* q = PT + (size_t)l * 16 * PW;
        double acc[K];
#pragma unroll
        for (int b = 0; b < K; ++b) acc[b] = 0.0;
#pragma unroll 2
        for (int p = 0; p < 16; ++p) {
            const double* r = q + p * PW;
            const double w = r[i] * r[kNP + j];
#pragma unroll
            for (int b = 0; b < K; ++b) acc[b] = __builtin_fma(w, r[2 * kNP + b], acc[b]);
        }
        // the 16 lanes of leaf l read all of its rows before any writes (one wave, in order)
        double* LM = PT + (size_t)l * 16 * PW;  // [16][K]
#pragma unroll
        for (int b = 0; b < K; ++b) LM[ln * K + b] = acc[b];
        if (active)
#pragma unroll
            for (int b = 0; b < K; ++b) n.upMult[((size_t)leafNode * kRank + ln) * K + b] = acc[b];
    }
    __syncthreads();
    double Rr[kRank];
    {
        const double* R2 = &P->R[threadIdx.x & 3][((threadIdx.x >> 2) & 15) * kRank];
#pragma unroll
        for (int rr = 0; rr < kRank; ++rr) Rr[rr] = threadIdx.x < 64 ? R2[rr] : 0.0;
    }
    {  // parent m, row r, child c (leaf slot 4 m + c, quadrant G[4 m + c] & 3)
        const int m = um, r = ur, c = uc;
        const double* x = PT + (size_t)(4 * m + c) * 16 * PW;
        double acc[K];
#pragma unroll
        for (int b = 0; b < K; ++b) acc[b] = 0.0;
#pragma unroll
        for (int rr = 0; rr < kRank; ++rr)
#pragma unroll
            for (int b = 0; b < K; ++b) acc[b] = __builtin_fma(Rc[rr], x[rr * K + b], acc[b]);
#pragma unroll
        for (int b = 0; b < K; ++b) acc[b] = quad_sum(acc[b]);
        if (c == 0) {
#pragma unroll
            for (int b = 0; b < K; ++b) {
                PM[(m * kRank + r) * K + b] = acc[b];
                n.upMult[((size_t)parentNode * kRank + r) * K + b] = acc[b];
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // the root: row r, parent m
        const int r = threadIdx.x >> 2, m = threadIdx.x & 3;
        const double* x = PM + (size_t)m * RK;
        double acc[K];
#pragma unroll
        for (int b = 0; b < K; ++b) acc[b] = 0.0;
#pragma unroll
        for (int rr = 0; rr < kRank; ++rr)
#pragma unroll
            for (int b = 0; b < K; ++b) acc[b] = __builtin_fma(Rr[rr], x[rr * K + b], acc[b]);
#pragma unroll
        for (int b = 0; b < K; ++b) acc[b] = quad_sum(acc[b]);
        if (m == 0)
#pragma unroll
            for (int b = 0; b < K; ++b) n.upMult[((size_t)rootNode * kRank + r) * K + b] = acc[b];
    }
}

template <int K, int U, int NR, bool FUSE, bool SYM, bool UP>
__device__ __forceinline__ void near_hs_group(const int g, const NearHsArgs& n, double* tab) {
    constexpr int KS = kStride<K>;
    constexpr int RW = kTabRow<K>;  // table row: x, y, the charges (padded)
    const int nl = n.nl;
    const int4* __restrict__ leafInfo = n.leafInfo;
    const int64_t* __restrict__ nearPtsPtr = n.nearPtsPtr;
    const uint16_t* __restrict__ nearLoc = n.nearLoc;
    const int64_t* __restrict__ nsPtr = n.nsPtr;
    const int* __restrict__ nsPts = n.nsPts;
    const int64_t* __restrict__ nearKOff = n.nearKOff;
    const double* __restrict__ E = n.E;
    const double* __restrict__ pxT = n.pxT;
    const double* __restrict__ pyT = n.pyT;
    const double* __restrict__ sigDiag = n.sigDiag;
    const HarmWeights& hw = n.hw;
    const double* __restrict__ fT = n.fT;
    const int* __restrict__ operm = n.operm;
    const int64_t obase = n.obase, ldo = n.ldo;
    const int flags = n.flags;
    const double scale = n.scale;
    double* __restrict__ out = n.out;
    const NearCorr& nc = n.nc;
    const bool nearOn = (flags & kStageNear) != 0;
    const bool fromIn = n.xin != nullptr;  // charges formed from the input (NearHsArgs)
    // the K weighted charges f = x sigma_s w of tree position p
    auto wcharges = [&](int64_t p, double (&f)[K]) {
        if (fromIn) {
            const double w = n.wT[p];
#pragma unroll
            for (int b = 0; b < K; ++b) f[b] = input_charge(n.xin, n.ldi, b, n.treeIn, n.perm, n.sigT, p) * w;
        } else {
            load_charges<K>(fT + (size_t)p * KS, f);
        }
    };
    // SYM: symmetric U storage (NearHsArgs::colDst; its own instance: the canonical
    // loop's registers would cost the directed kernel a wave per SIMD); the partner
    // products within the group go to LDS slots after the table, 16 rows x K each
    const bool sym = SYM && nearOn;
    double* dslot = tab + (size_t)n.nsMax * RW;
    if (nearOn) {
        const int64_t r0 = nsPtr[g];
        const int nr = (int)(nsPtr[g + 1] - r0);
        for (int i = threadIdx.x; i < nr; i += blockDim.x) {
            const int64_t p = nsPts[r0 + i];
            double* row = tab + (size_t)i * RW;
            row[0] = pxT[p];
            row[1] = pyT[p];
            double f[K];
            wcharges(p, f);
#pragma unroll
            for (int v = 0; v < K; ++v) row[2 + v] = f[v];
        }
    }
#ifdef ANISO_NEAR_SYM_ATOMIC
    if (sym)
        for (int i = threadIdx.x; i < 256 * K; i += blockDim.x) dslot[i] = 0.0;
#endif
    __syncthreads();
    const int gl = threadIdx.x & 15;
    const int li = g * 16 + (int)(threadIdx.x >> 4);
    const bool active = li < nl;
    int4 info = make_int4(0, 0, 0, 0);
    int64_t pb = 0, koff = 0;
    if (active) {
        info = leafInfo[li];
        pb = nearPtsPtr[li];
        koff = nearKOff[li];
    }
    const int nT = info.z;
    // the directed columns (symmetric storage: the canonical blocks follow them)
    const int S = !nearOn ? 0 : sym && active ? n.nearSym[li].x : info.w;
    const int64_t tb = info.y;
    const int nq = (nT + 3) >> 2;
    const int cstr = 2 * nq;
    const int rq = gl & 3, cph = gl >> 2;  // 4 lanes per column, 4 column phases
    const bool rowOk = active && rq < nq;
    double tx[4], ty[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int t = min(4 * rq + j, max(nT - 1, 0));  // padded rows: E is zero there
        tx[j] = rowOk ? pxT[tb + t] : 0.0;
        ty[j] = rowOk ? pyT[tb + t] : 0.0;
    }
    double a[4][K];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < K; ++i) a[j][i] = 0.0;
    if (rowOk) {
        const dbl2* kc = reinterpret_cast<const dbl2*>(E + koff) + 2 * rq;
        // U columns per lane and step: their E quads (16 B x 2) and table rows
        auto fetch = [&](int c0, dbl2 (&kk)[U][2], int (&ix)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int sc = c0 + u * 4;
                const bool ok = sc < S;
                const dbl2* p = kc + (size_t)min(sc, S - 1) * cstr;
                kk[u][0] = ok ? __builtin_nontemporal_load(p) : dbl2{0.0, 0.0};
                kk[u][1] = ok ? __builtin_nontemporal_load(p + 1) : dbl2{0.0, 0.0};
                ix[u] = nearLoc[pb + min(sc, S - 1)];
            }
        };
        auto step = [&](const dbl2 (&kk)[U][2], const int (&ix)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double* row = tab + (size_t)ix[u] * RW;
                const double sx = row[0], sy = row[1];
                double xw[K];
#pragma unroll
                for (int b = 0; b < K; ++b) xw[b] = hw.hw[b] * row[2 + b];
                const double e4[4] = {kk[u][0].x, kk[u][0].y, kk[u][1].x, kk[u][1].y};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double dy = sy - ty[j];
                    hm_entry<K, true, NR>(e4[j], sx - tx[j], dy * dy, xw, a[j]);
                }
            }
        };
        for (int c0 = cph; c0 < S; c0 += U * 4) {
            dbl2 kk[U][2];
            int ix[U];
            fetch(c0, kk, ix);
            step(kk, ix);
        }
    }
    if constexpr (SYM) if (sym && active) {
        // canonical partner blocks (the U pairs this leaf stores, bbfmm.h:1081-1099): one
        // read of E(t, s) serves both ends -- this leaf's rows as above, and the
        // partner's point s, whose product sums the leaf's rows (in-lane, then over the
        // row quads by DPP: every lane of an active leaf takes part, padded rows read 0)
        // and goes to the pair's LDS slot or to the partner's partial slot (colDst).
        // The reversed direction has cos = -c: (-1)^b on the leaf's charges, (-1)^i on
        // the product (as hm_entry2 in the cluster M2L).  UC columns in flight per lane.
        constexpr int UC = 2;
        double xa[4][K];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * rq + j;
            const double* row = tab + (size_t)(n.selfRow[li] + min(t, max(nT - 1, 0))) * RW + 2;
#pragma unroll
            for (int b = 0; b < K; ++b) xa[j][b] = t < nT ? ((b & 1) ? -hw.hw[b] : hw.hw[b]) * row[b] : 0.0;
        }
        const dbl2* kc = reinterpret_cast<const dbl2*>(E + koff) + 2 * rq;
        const int S1 = n.nearSym[li].y;
        const int* __restrict__ dst = n.colDst + pb;
        for (int c0 = S + cph; c0 < S1; c0 += UC * 4) {
            dbl2 kk[UC][2];
            int ix[UC], dd[UC];
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                const int sc = min(c0 + u * 4, S1 - 1);
                const bool ok = c0 + u * 4 < S1 && rq < nq;
                const dbl2* p = kc + (size_t)sc * cstr;
                kk[u][0] = ok ? __builtin_nontemporal_load(p) : dbl2{0.0, 0.0};
                kk[u][1] = ok ? __builtin_nontemporal_load(p + 1) : dbl2{0.0, 0.0};
                ix[u] = nearLoc[pb + sc];
                dd[u] = dst[sc];
            }
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                if (c0 + u * 4 >= S1) break;  // uniform over the quad (one column phase)
                const double* row = tab + (size_t)ix[u] * RW;
                const double sx = row[0], sy = row[1];
                double xw[K], ob[K];
#pragma unroll
                for (int b = 0; b < K; ++b) {
                    xw[b] = hw.hw[b] * row[2 + b];
                    ob[b] = 0.0;
                }
                const double e4[4] = {kk[u][0].x, kk[u][0].y, kk[u][1].x, kk[u][1].y};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double dy = sy - ty[j];
                    hm_entry2<K, NR>(e4[j], sx - tx[j], dy * dy, xw, xa[j], a[j], ob);
                }
#pragma unroll
                for (int i = 0; i < K; ++i) ob[i] = quad_sum(ob[i]);  // the leaf's rows: over the row quads
                // lane rq of the quad stores products i = rq (and rq + 4)
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    if ((i & 3) != rq) continue;
                    const double v = (i & 1) ? -ob[i] : ob[i];
#ifdef ANISO_NEAR_SYM_ATOMIC
                    if (dd[u] < 0) atomicAdd(dslot + (size_t)(~dd[u]) * K + i, v);
#else
                    if (dd[u] < 0) dslot[(size_t)(~dd[u]) * K + i] = v;
#endif
                    else n.nearPart[(size_t)dd[u] * K + i] = hw.om[i] * v;
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)  // sum over the column phases
#pragma unroll
        for (int i = 0; i < K; ++i) {
            double v = a[j][i];
            v += dpp_f64<0x124>(v);  // row_ror:4
            v += dpp_f64<0x128>(v);  // row_ror:8
            a[j][i] = v;
        }
    if (sym) __syncthreads();  // every partner product of the group is in LDS
    double fq[K];  // the lane's point's weighted charges (the fused up tail's P2M)
#pragma unroll
    for (int i = 0; i < K; ++i) fq[i] = 0.0;
    if (rowOk) {  // lane (rq, cph) finishes row 4 rq + cph: one pass with every lane active
        const int t = 4 * rq + cph;
        double av[K];
#pragma unroll
        for (int i = 0; i < K; ++i) av[i] = cph == 0 ? a[0][i] : cph == 1 ? a[1][i] : cph == 2 ? a[2][i] : a[3][i];
#ifdef ANISO_NEAR_SYM_ATOMIC
        if (sym && t < nT) {
            const double* d = dslot + ((size_t)(li & 15) * 16 + t) * K;
#pragma unroll
            for (int i = 0; i < K; ++i) av[i] += d[i];
        }
        if (false) {
#else
        if (sym && t < nT) {  // the products this group's smaller-id partners left for the row, in slot order
#endif
            const int q1 = n.grpInPtr[li + 1];
            for (int q = n.grpInPtr[li]; q < q1; ++q) {
                const double* d = dslot + ((size_t)n.grpIn[q] * 16 + t) * K;
#pragma unroll
                for (int i = 0; i < K; ++i) av[i] += d[i];
            }
        }
        if (t < nT) {
            const int64_t k = tb + t;
            double f[K];
            wcharges(k, f);
#pragma unroll
            for (int i = 0; i < K; ++i) fq[i] = f[i];
            const double sd = nearOn ? sigDiag[k] : 0.0;
            const int64_t oi = out_index(operm, obase, k);
            double cr[K];  // FUSE: k_corr's contribution (d = 1), its neighbour charges from the table
            if constexpr (FUSE) {
                const uint16_t* rw = nc.rows + ((size_t)li * 16 + t) * 9;
                auto cval = [&](int64_t p, int r) {
                    return fromIn ? input_charge(n.xin, n.ldi, r, n.treeIn, n.perm, n.sigT, p)
                                  : nc.cT[(size_t)p * KS + r];
                };
                corr_point<1, K>(nc.perm[k], nc.P, nc.iperm, cval, nc.Wc, nc.Wm, flags,
                                 [&](int q9, int, int, double (&fc)[K]) {
                                     const double* row = tab + (size_t)rw[q9] * RW + 2;
#pragma unroll
                                     for (int b = 0; b < K; ++b) fc[b] = row[b];
                                 },
                                 cr);
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) cr[i] = 0.0;
            }
#pragma unroll
            for (int i = 0; i < K; ++i)
                out[(size_t)i * ldo + oi] =
                    __builtin_fma(hw.om[i] * scale, __builtin_fma(hw.dw[i] * sd, f[i], av[i]), cr[i] * scale);
        }
    }
    if constexpr (UP) near_up_tail<K>(g, active, nT, tb, info.x, n, fq, tab);
}

// the staged near field's LDS: the source table, and with symmetric U storage the
// group's partner product slots (16 rows x K each)
template <int K>
static size_t near_hs_lds(const NearHsArgs& n) {
    const size_t tab = (size_t)n.nsMax * kTabRow<K> * sizeof(double) +
                       (n.colDst ? (size_t)n.grpSlots * 16 * K * sizeof(double) : 0);
    return std::max(tab, n.upMult ? near_up_lds_doubles(K) * sizeof(double) : (size_t)0);  // the up tail reuses the table
}

// W4: capped at 128 VGPRs (4 waves per SIMD; ANISO_NEAR_WPE=4)
#ifndef ANISO_NEAR_SYM_WPE
#define ANISO_NEAR_SYM_WPE 1
#endif
template <int K, int U, int NR, bool FUSE, bool W4 = false, bool SYM = false, bool UP = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W4 ? 4 : SYM ? ANISO_NEAR_SYM_WPE : 1))) k_near_hs(NearHsArgs n) {
    extern __shared__ double tab[];
    // the fused top-of-tree launch's counters (the bottom tier launch that zeroes them is skipped)
    if (n.zeroCnt && blockIdx.x == 0 && threadIdx.x <= kMaxTopTiers) n.zeroCnt[threadIdx.x] = 0u;
    near_hs_group<K, U, NR, FUSE, SYM, UP>(n.grpList ? n.grpList[blockIdx.x] : (int)blockIdx.x, n, tab);
}


// ----------------------------------------------------------------- launchers

#define ANISO_HM_DISPATCH_K(k, CALL)                                                                    \
    switch (k) {                                                                                        \
        case 2: { constexpr int KK = 2; CALL; } break;                                                  \
        case 4: { constexpr int KK = 4; CALL; } break;                                                  \
        case 5: { constexpr int KK = 5; CALL; } break;                                                  \
        case 8: { constexpr int KK = 8; CALL; } break;                                                  \
        default: throw std::invalid_argument("harmonic apply: unsupported block count " + std::to_string(k)); \
    }

// per-target M2L (ANISO_HM_CLUSTER=0): two Newton steps in 1/r (full fp64), 4 waves
// per SIMD (measured best, r01e)
void launch_m2l_hm(int K, int ntgt, const int* tgt, const int64_t* ptr, const int* src, const int* blk, const double* E,
                   const double* ncx, const double* ncy, const double* nrx, const double* nry, const Params* P,
                   const HarmWeights& hw, const double* mult, double* local, hipStream_t s) {
    if (ntgt <= 0) return;
    const unsigned nb = blocks_for((int64_t)ntgt * kWave, 256);
    ANISO_HM_DISPATCH_K(K, (k_m2l_hm<KK, 2, 2, 4><<<nb, 256, 0, s>>>(ntgt, 0, tgt, ptr, src, blk, E, ncx, ncy, nrx, nry,
                                                                      P, hw, mult, local)));
    HIP_LAUNCH_CHECK();
}

// clustered M2L (the default): 4 waves per cluster of <= 64 targets (512 / 768
// threads, 2 waves per SIMD, 128-target clusters, a software-pipelined stream and an
// XCD-contiguous cluster order all measured equal or slower, r01e-r01j), 3 waves per
// SIMD; 1/r = v_rsq_f64 + ONE Newton step (~1e-13 relative per entry, 4 % faster
// than two; the reduced-precision choice is tested at 1M points)
size_t m2l_hc_lds(int K, int maxCl, int depth, bool xl, int nw) {
    size_t b = (size_t)maxCl * kRank * K * sizeof(double);
    if (depth == 0 || xl) b += (size_t)nw * kRank * K * sizeof(double);  // each wave's weighted target multipole
    if (depth == 0) return b;
    const size_t slot = 2048 + (size_t)kRank * K * 8 + 32;
    return b + (size_t)nw * depth * slot;
}

// the ring form (k_m2l_hcr, the default) and its depth: ANISO_HM_RING=0 restores the
// one-block-in-flight form (A/B runs), ANISO_HM_RING=2..4 sets the depth
int hm_ring_depth() {
    const char* e = std::getenv("ANISO_HM_RING");
    const int v = e ? std::atoi(e) : 0;
    return v == 0 ? 0 : std::max(2, std::min(4, v));
}

// the ring form's target multipole: 1 in LDS (3 waves per SIMD), 0 in VGPRs (2 waves
// per SIMD), -1 the ring form not used.  By default the LDS form where three
// workgroups per CU fit in LDS with it (small clusters: shards); elsewhere the
// one-block-in-flight form, which keeps 3 waves per SIMD there (r03m: at 64-target
// clusters the ring's LDS allows 2 workgroups per CU and is 5-7 % slower).
// ANISO_HM_RING_XL=0 / 1 forces the VGPR / LDS form.
// K = 8 (aniso.m with more than 5 blocks) keeps the one-block-in-flight form: both
// ring forms spill there, and a scratch store inside the stream would break the
// counted vmcnt waits (stores retire out of order with the LDS-DMA loads).
int hm_ring_xl(int K, int maxCl, int depth) {
    if (K > kRingMaxK) return -1;
    if (const char* e = std::getenv("ANISO_HM_RING_XL")) return std::atoi(e) != 0 ? 1 : 0;
    return 3 * m2l_hc_lds(K, maxCl, depth, true, 4) <= 160 * 1024 ? 1 : -1;
}

#define ANISO_HM_DISPATCH_RING(d, CALL)                                            \
    switch (d) {                                                                   \
        case 0: { constexpr int DD = 0; CALL; } break;                             \
        case 2: { constexpr int DD = 2; CALL; } break;                             \
        case 3: { constexpr int DD = 3; CALL; } break;                             \
        case 4: { constexpr int DD = 4; CALL; } break;                             \
        default: throw std::invalid_argument("harmonic M2L: bad ring depth");      \
    }

// The one-block cluster form's occupancy, ANISO_HM_WPE:
// 3 = 3 waves per SIMD in 4-wave workgroups; 6 = 3 waves per SIMD in 6-wave
// workgroups (2 per CU); 4 = 4 waves per SIMD (<= 128 VGPRs, m2l_hc_cluster<LR>) in
// 4-wave workgroups, which needs 4 of them per CU in LDS (small clusters: shards);
// 8 = the LR form in 8-wave workgroups, 2 per CU.  The 4-wave-per-SIMD forms
// measured slower (r03lr: a rank of 8 0.300 against 0.269 ms fused; one GPU with
// 8-wave workgroups 1.300 against 1.324 ms, but 1.343 beside the 4-wave near field).
// Default: 3 waves per SIMD, in 4-wave workgroups where 3 fit per CU in LDS
// (shm4: the launch's LDS per workgroup with 4 waves), else in 6-wave ones (the halo
// form's 64-target clusters: ~72 KB).
static int hm_form(int K, int wpe, size_t shm4) {
    if ((wpe == 4 || wpe == 8) && K <= kRingMaxK) return wpe;
    if (wpe == 3 || wpe == 6) return wpe;
    return 3 * shm4 <= 160 * 1024 ? 3 : 6;
}

static int hm_threads(int form) { return form == 8 ? 512 : form == 6 ? 384 : 256; }
static int hm_waves(int form) { return hm_threads(form) / kWave; }

template <typename F>
static void set_lds(F f, size_t shm) {
    if (shm > 65536) {  // clusters of up to 64 targets need more than the default 64 KB
        const hipError_t e =
            hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
    }
}

// clustered M2L (the default): 4 waves per cluster of <= 64 targets (512 / 768
// threads, 2 waves per SIMD, 128-target clusters, a software-pipelined stream and an
// XCD-contiguous cluster order all measured equal or slower, r01e-r01j), 3 waves per
// SIMD; 1/r = v_rsq_f64 + ONE Newton step (~1e-13 relative per entry, 4 % faster
// than two; the reduced-precision choice is tested at 1M points)
void launch_m2l_hc(int K, int ncl, int maxCl, const HcArgs& a, hipStream_t s) {
    if (ncl <= 0) return;
    const int depth = a.geo && K <= kRingMaxK ? a.ring : 0;
    const bool xl = a.ringXL;
    size_t shm = m2l_hc_lds(K, maxCl, depth, xl, 4);
    const int form = depth == 0 ? hm_form(K, a.wpe, shm) : 3;
    if (form != 3) shm = m2l_hc_lds(K, maxCl, depth, xl, hm_waves(form));
    if (shm > 160 * 1024) throw std::invalid_argument("harmonic M2L: a cluster and its halo exceed the LDS");
    if (a.wmax) {  // the deterministic sums: the one-block 3-wave-per-SIMD forms (whatever the ring knob says)
        const int fd = hm_form(K, 0, shm);
        const size_t shd = m2l_hc_lds(K, maxCl, 0, false, hm_waves(fd));
        ANISO_HM_DISPATCH_K(K, ({
            auto f = fd == 6 ? k_m2l_hc<KK, 1, 6, true> : k_m2l_hc<KK, 1, 3, true>;
            set_lds(f, shd);
            f<<<ncl, hm_threads(fd), shd, s>>>(a);
        }));
        HIP_LAUNCH_CHECK();
        return;
    }
    ANISO_HM_DISPATCH_K(K, ANISO_HM_DISPATCH_RING(depth, ({
        if constexpr (DD == 0 || KK > kRingMaxK) {
            auto f = form == 6 ? k_m2l_hc<KK, 1, 6> : k_m2l_hc<KK, 1, 3>;
            if constexpr (KK <= kRingMaxK) {
                if (form == 4) f = k_m2l_hc<KK, 1, 4>;
                if (form == 8) f = k_m2l_hc<KK, 1, 8>;
            }
            set_lds(f, shm);
            f<<<ncl, hm_threads(form), shm, s>>>(a);
        } else {
            auto f = xl ? k_m2l_hcr<KK, 1, DD, true, 3> : k_m2l_hcr<KK, 1, DD, false, 2>;
            set_lds(f, shm);
            f<<<ncl, 256, shm, s>>>(a);
        }
    })));
    HIP_LAUNCH_CHECK();
}

// The deterministic sums' bounds (hc_det_scale): W per node, the largest |E|
template <int K>
__global__ void __launch_bounds__(256) k_node_wmax(int nnodes, const double* __restrict__ mult, HarmWeights hw,
                                                   double* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (node, column): 16 lanes per node
    const int64_t n = t >> 4;
    double w = 0.0;
    if (n < nnodes) {
        const double* m = mult + (size_t)t * K;
#pragma unroll
        for (int b = 0; b < K; ++b) w += fabs(hw.hw[b] * m[b]);
    }
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) w = fmax(w, __shfl_xor(w, off));
    if (n < nnodes && (t & 15) == 0) out[n] = w;
}

__global__ void __launch_bounds__(256) k_abs_max(int64_t n, const double* __restrict__ x,
                                                 unsigned long long* __restrict__ out) {
    double m = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        m = fmax(m, fabs(x[i]));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    // non-negative doubles order as their bit patterns
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

void launch_node_wmax(int K, int nnodes, const double* mult, const HarmWeights& hw, double* out, hipStream_t s) {
    if (nnodes <= 0) return;
    const int nb = (int)(((int64_t)nnodes * 16 + 255) / 256);
    ANISO_HM_DISPATCH_K(K, (k_node_wmax<KK><<<nb, 256, 0, s>>>(nnodes, mult, hw, out)));
    HIP_LAUNCH_CHECK();
}

void launch_abs_max(int64_t n, const double* x, double* out, hipStream_t s) {
    const hipError_t e = hipMemsetAsync(out, 0, sizeof(double), s);
    if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
    if (n <= 0) return;
    const int nb = (int)std::min<int64_t>(4096, (n + 255) / 256);
    k_abs_max<<<nb, 256, 0, s>>>(n, x, reinterpret_cast<unsigned long long*>(out));
    HIP_LAUNCH_CHECK();
}

bool top_fused_enabled() {
#ifdef ANISO_NO_TOP_FUSED
    return false;
#else
    return true;
#endif
}

void launch_top_m2l_hc(int K, int ncl, int maxCl, const UpArgs& u, const TopArgs& t0, const HcArgs& a,
                       const NearHsArgs* near, hipStream_t s) {
    if (t0.ntier < 2 || t0.ntier > kMaxTopTiers || t0.blk0[t0.ntier] != t0.nUp)
        throw std::invalid_argument("fused top-of-tree launch: bad tier layout");
    if (!t0.err) throw std::invalid_argument("fused top-of-tree launch: no time-out flag");
    const int depth = a.geo && K <= kRingMaxK ? a.ring : 0;
    if (near && (depth != 0 || near->nl <= 0))
        throw std::invalid_argument("fused top-of-tree launch: the near field rides only with the one-block M2L");
    if (near && near->colDst)
        throw std::invalid_argument("fused top-of-tree launch: the near field rides only with directed U storage");
    const bool xl = a.ringXL;
    TopArgs t = t0;
    t.nCl = ncl;
    const NearHsArgs n = near ? *near : NearHsArgs{};
    const unsigned nb = (unsigned)(t.nUp + ncl) + (near ? (unsigned)((near->nl + 15) / 16) : 0u);
    ANISO_HM_DISPATCH_K(K, ANISO_HM_DISPATCH_RING(depth, ({
        size_t shm = std::max(m2l_hc_lds(KK, maxCl, depth, xl, 4), up_tier_lds(u.maxTask, KK));
        if (near) shm = std::max(shm, near_hs_lds<KK>(*near));
        const int form = DD == 0 && !near ? hm_form(KK, a.wpe, shm) : 3;
        if (form != 3) shm = std::max(shm, m2l_hc_lds(KK, maxCl, depth, xl, hm_waves(form)));
        if (shm > 160 * 1024) throw std::invalid_argument("fused top-of-tree launch: a cluster and its halo exceed the LDS");
        // the ring form with its target multipole in VGPRs needs ~216 of them at K = 5
        if constexpr (DD == 0 || KK > kRingMaxK) {
            auto f = near ? (t.trace ? k_top_m2l_hc<KK, 1, 3, 0, false, true, true>
                                     : k_top_m2l_hc<KK, 1, 3, 0, false, false, true>)
                          : (t.trace ? k_top_m2l_hc<KK, 1, 3, 0, false, true> : k_top_m2l_hc<KK, 1, 3, 0, false>);
            if (form == 6) f = t.trace ? k_top_m2l_hc<KK, 1, 6, 0, false, true> : k_top_m2l_hc<KK, 1, 6, 0, false>;
            if constexpr (KK <= kRingMaxK) {
                if (form == 4) f = t.trace ? k_top_m2l_hc<KK, 1, 4, 0, false, true> : k_top_m2l_hc<KK, 1, 4, 0, false>;
                if (form == 8) f = t.trace ? k_top_m2l_hc<KK, 1, 8, 0, false, true> : k_top_m2l_hc<KK, 1, 8, 0, false>;
            }
            set_lds(f, shm);
            f<<<nb, hm_threads(form), shm, s>>>(u, t, a, n);
        } else {
            auto f = xl ? (t.trace ? k_top_m2l_hc<KK, 1, 3, DD, true, true> : k_top_m2l_hc<KK, 1, 3, DD, true>)
                        : (t.trace ? k_top_m2l_hc<KK, 1, 2, DD, false, true> : k_top_m2l_hc<KK, 1, 2, DD, false>);
            set_lds(f, shm);
            f<<<nb, 256, shm, s>>>(u, t, a, n);
        }
    })));
    HIP_LAUNCH_CHECK();
}

// near field: 16 lanes per leaf for leaves <= 16 points (4 leaves per wave), a wave
// per leaf otherwise; 4 source columns in flight per lane (2 and 8, XCD-contiguous
// leaves and leaf clusters measured slower, r01h); 1/r to full fp64 (two Newton steps).
// The staged kernel k_near_hs takes 2 columns per step: 121 VGPRs, so 4 waves per
// SIMD fit beside its 32 KB source table (standalone 3-6 % faster than 4 columns at 3
// waves, r04ak)
static bool near_hs_staged(int nl, int maxLeaf, int nsMax, const uint16_t* nearLoc) {
    return nl > 0 && maxLeaf <= 16 && nsMax > 0 && nearLoc && (size_t)nsMax * kTabRow<8> * sizeof(double) <= 64 * 1024;
}


bool near_hs_fusable(int nl, int maxLeaf, int nsMax, const uint16_t* nearLoc, const NearCorr* corr, int flags) {
    return near_hs_staged(nl, maxLeaf, nsMax, nearLoc) && corr && corr->rows && (flags & kStageNear);
}

bool launch_near_hm(int K, int nl, int maxLeaf, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts,
                    const int64_t* nearKOff, const double* E, const double* pxT, const double* pyT,
                    const double* sigDiag, const HarmWeights& hw, const double* fT, const int* operm, int64_t obase,
                    int64_t ldo, int flags, double scale, double* out, const uint16_t* nearLoc, const int64_t* nsPtr,
                    const int* nsPts, int nsMax, const NearCorr* corr, int wpe, hipStream_t s, const NearHsArgs* in) {
    if (nl <= 0) return false;
    if (near_hs_staged(nl, maxLeaf, nsMax, nearLoc)) {  // sources staged in LDS (k_near_hs)
        unsigned ng = (unsigned)((nl + 15) / 16);
        // the corrections ride along when the table is loaded (near field on)
        const bool fuse = near_hs_fusable(nl, maxLeaf, nsMax, nearLoc, corr, flags);
        NearHsArgs n{nl, nsMax, leafInfo, nearPtsPtr, nearLoc, nsPtr, nsPts, nearKOff, E, pxT, pyT, sigDiag, hw,
                     fT, operm, obase, ldo, flags, scale, out, fuse ? *corr : NearCorr{}};
        if (in && in->xin) {  // charges from the input (the near field beside the up pass)
            if (!fuse) throw std::invalid_argument("near field from the input: only with its fused corrections");
            n.xin = in->xin;
            n.ldi = in->ldi;
            n.treeIn = in->treeIn;
            n.perm = in->perm;
            n.sigT = in->sigT;
            n.wT = in->wT;
        }
        if (in && in->upMult) {  // the bottom up tier in the near field (the caller checked near_up_fits)
            if (!fuse || in->colDst)
                throw std::invalid_argument("near field with the up tier: not the staged directed kernel with its table");
            n.upMult = in->upMult;
            n.upGrp = in->upGrp;
            n.upP = in->upP;
            n.upNcx = in->upNcx;
            n.upNcy = in->upNcy;
            n.upNrx = in->upNrx;
            n.upNry = in->upNry;
            n.zeroCnt = in->zeroCnt;
        }
        if (in && in->grpList) {  // a subset of the groups
            n.grpList = in->grpList;
            n.ngrp = in->ngrp;
            ng = (unsigned)in->ngrp;
            if (ng == 0) return fuse;
        }
        if (in && in->colDst) {  // symmetric U storage (the column lists passed are its own)
            if (!in->nearSym || !in->selfRow || !in->nearPart || !in->grpInPtr)  // grpIn: may be empty
                throw std::invalid_argument("symmetric staged near field: missing lists");
            n.nearSym = in->nearSym;
            n.colDst = in->colDst;
            n.selfRow = in->selfRow;
            n.nearPart = in->nearPart;
            n.grpInPtr = in->grpInPtr;
            n.grpIn = in->grpIn;
            n.grpSlots = in->grpSlots;
        }
        ANISO_HM_DISPATCH_K(K, ({
            const size_t shm = near_hs_lds<KK>(n);
            auto f = n.colDst ? (fuse ? k_near_hs<KK, 4, 2, true, false, true> : k_near_hs<KK, 4, 2, false, false, true>)
                     // with the up tail: the 4-wave form (<= 128 VGPRs)
                     : fuse ? (n.upMult ? k_near_hs<KK, 2, 2, true, true, false, true>
                               : wpe == 4 ? k_near_hs<KK, 2, 2, true, true> : k_near_hs<KK, 2, 2, true>)
                            : (wpe == 4 ? k_near_hs<KK, 2, 2, false, true> : k_near_hs<KK, 2, 2, false>);
            f<<<ng, 256, shm, s>>>(n);
        }));
        HIP_LAUNCH_CHECK();
        return fuse;
    }
#define ANISO_NEAR_HM(G)                                                                                      \
    ANISO_HM_DISPATCH_K(K, (k_near_hm<KK, G, 4, 2><<<blocks_for((int64_t)nl * G, 256), 256, 0, s>>>(           \
                               nl, leafInfo, nearPtsPtr, nearPts, nearKOff, E, pxT, pyT, sigDiag, hw, fT, operm, \
                               obase, ldo, flags, scale, out)))
    if (in && in->colDst) throw std::invalid_argument("symmetric near storage needs the staged near field");
    if (in && in->grpList) throw std::invalid_argument("a near-field group subset needs the staged near field");
    if (maxLeaf <= 16) {
        ANISO_NEAR_HM(16);
    } else {
        ANISO_NEAR_HM(64);
    }
#undef ANISO_NEAR_HM
    HIP_LAUNCH_CHECK();
    return false;
}

}  // namespace aniso
