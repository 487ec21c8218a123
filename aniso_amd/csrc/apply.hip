// apply.hip -- the apply kernels (one mode-apply of the anisotropic RTE operator,
// AnisoWrapper.cpp:92-136), for K right-hand sides at once.
//
// Reference behaviour (file:line under lowrank/aniso):
//   up pass      bbfmm.h:825-861          (P2M leaf transfer, M2M)
//   down pass    bbfmm.h:1041-1129        (M2L over V/X, L2L, U/W near, L2P)
//   corrections  KernelFactory.cpp:445-478, 662-709, 828-860
//   block caller aniso.m:139-157          (mforward: 9 modes x 5 blocks)
//
// Batching.  K right-hand sides share one read of every cached
// operator.  The up pass computes the multipoles of K *base* vectors; each mode's
// kernels apply a K x K mix to them on the fly (rhs i = sum_b mix[i][b] base b), so
// the block operator of aniso.m streams each mode's operators once for all its
// right-hand sides.  The far field is linear in the locals and L2L/L2P do not
// depend on the mode, so locals and transposed near products accumulate over the
// modes of a call and the down pass runs once.
//
// Layouts (K fastest): fT, cT [N][KS] tree order (KS = K rounded up to even); mult, local [node][16][K];
// M2L partials [slot][16][K]; near partials [column][K]; outputs [K][ldo].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "corr_point.hpp"
#include "device_common.hpp"
#include "host.hpp"
#include "up_task.hpp"

namespace aniso {


template <int K>
struct MixK {
    double c[K][K];  // rhs i = sum_b c[i][b] * base b
};

template <int K>
__device__ __forceinline__ void mix_apply(const MixK<K>& m, const double* base, double* v) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double a = 0.0;
#pragma unroll
        for (int b = 0; b < K; ++b) a += m.c[i][b] * base[b];
        v[i] = a;
    }
}

// The same with a term's mix from the device mode table.
template <int K>
__device__ __forceinline__ void mix_apply_t(const ModeArgs& m, const double* base, double* v) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double a = 0.0;
#pragma unroll
        for (int b = 0; b < K; ++b) a += m.mix[i][b] * base[b];
        v[i] = a;
    }
}


// fT[k][b] = c w_T[k] (FMM and stencil charges), cT[k][b] = c (singular term).
// The up pass forms them inside its P2M; this kernel covers a tree without
// up-pass tiers (a lone leaf).
template <int K>
__global__ void k_prepare(int64_t N, const double* __restrict__ xin, int64_t ldi, int treeIn,
                          const int* __restrict__ perm, const double* __restrict__ sigT, const double* __restrict__ wT,
                          double* __restrict__ fT, double* __restrict__ cT) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
#pragma unroll
    for (int b = 0; b < K; ++b) {
        const double c = input_charge(xin, ldi, b, treeIn, perm, sigT, k);
        fT[k * kStride<K> + b] = c * wT[k];
        cT[k * kStride<K> + b] = c;
    }
}

// y[i] = x[i] - a[i] on the owned slice, for each right-hand side
// (forwardOperator u - K(sigma_s u), main.cpp:125-136; aniso.m x - mforward(x)).
__global__ void k_sub_slice(int64_t n, int nrhs, const double* __restrict__ x, int64_t ldx,
                            const double* __restrict__ a, int64_t lda, double* __restrict__ y, int64_t ldy) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * nrhs) return;
    const int64_t r = i / n, j = i - r * n;
    y[r * ldy + j] = x[r * ldx + j] - a[r * lda + j];
}

// ----------------------------------------------------------------- up pass

// One partial task of the upper multipoles (Plan::xUpTask): this rank's
// tier-0 roots under one node A two levels above them.  M2M (bbfmm.h:855-859) of the
// roots to the mid level and to A, then A's contribution to each ancestor up to the
// topmost level an M2L reads, one transfer matrix per level; each share an M2L reads is
// a record, stored into rec and into every peer part.  sm: up_partial_lds<K>() doubles
// of LDS; 256 threads.
constexpr int kUpMaxPeers = 63;  // peer parts whose offsets the partial task holds in LDS
template <int K>
constexpr int up_partial_lds() {
    return Plan::kUpTaskInts + (kUpMaxPeers + 1) + 4 * kRank * kRank + 16 * kRank * K +
           (5 + Plan::kUpChainMax) * kRank * K;
}
// stage (tails): the roots from the write-through staging copies, slot q at
// stage + q * RK, read with sc1 loads (no acquire fence; MI355X_MICROARCH.md, the
// last-adder hand-off with write-through payload); else from mult by node id.
// Every record is formed in LDS first and stored in one final pass: a barrier
// between the levels then waits for LDS work only, not for the records' global
// stores (with a store pass per level the task took ~30 us under the near field).
template <int K>
__device__ __forceinline__ void up_partial_task(const int* __restrict__ tk, const Params* __restrict__ P,
                                                const double* __restrict__ mult, double* __restrict__ rec, int nPeer,
                                                const int64_t* __restrict__ peerOff, double* __restrict__ buf,
                                                double* sm, double* stage = nullptr) {
    constexpr int RK = kRank * K;
    constexpr int NI = Plan::kUpTaskInts;
    int* T = reinterpret_cast<int*>(sm);                // NI ints (NI doubles reserved)
    int64_t* PO = reinterpret_cast<int64_t*>(sm + NI);  // the peer parts' offsets
    double* Rm = sm + NI + kUpMaxPeers + 1;             // R[q][r * 16 + rr]: row r of quadrant q's M2M
    double* X = Rm + 4 * kRank * kRank;                 // the roots, slot 4 q1 + q0
    double* Mid = X + 16 * RK;                          // the 4 mid-level records
    double* C0 = Mid + 4 * RK;                          // A's share, then its contributions up the chain
    for (int i = threadIdx.x; i < NI; i += blockDim.x) T[i] = tk[i];
    for (int i = threadIdx.x; i < nPeer; i += blockDim.x) PO[i] = peerOff[i];
    for (int i = threadIdx.x; i < 4 * kRank * kRank; i += blockDim.x) Rm[i] = (&P->R[0][0])[i];
    if (stage) {  // slot q's root at stage + q RK (absent slots: never staged, read as 0 below)
        for (int i = threadIdx.x; i < 16 * RK; i += blockDim.x)
            X[i] = __hip_atomic_load(stage + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        for (int i = threadIdx.x; i < 16 * RK; i += blockDim.x)
            if (T[i / RK] < 0) X[i] = 0.0;
    } else {
        __syncthreads();
        for (int i = threadIdx.x; i < 16 * RK; i += blockDim.x) {
            const int r = T[i / RK];
            X[i] = r >= 0 ? mult[(size_t)r * RK + i % RK] : 0.0;
        }
    }
    __syncthreads();
    // parent entry (r, b) = sum over quadrants q and rows rr of R[q][r, rr] child_q[rr, b]
    auto m2m = [&](const double* child, int q, int r, int b, double acc) {
        const double* R = Rm + q * kRank * kRank + r * kRank;
#pragma unroll
        for (int rr = 0; rr < kRank; ++rr) acc += R[rr] * child[rr * K + b];
        return acc;
    };
    for (int it = threadIdx.x; it < 4 * RK; it += blockDim.x) {
        const int q1 = it / RK, e = it - q1 * RK, r = e / K, b = e - r * K;
        double acc = 0.0;
        for (int q0 = 0; q0 < 4; ++q0) acc = m2m(X + (4 * q1 + q0) * RK, q0, r, b, acc);
        Mid[it] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < RK; e += blockDim.x) {
        const int r = e / K, b = e - r * K;
        double acc = 0.0;
        for (int q1 = 0; q1 < 4; ++q1) acc = m2m(Mid + q1 * RK, q1, r, b, acc);
        C0[e] = acc;
    }
    const int nc = T[21];
    for (int c = 0; c < nc; ++c) {
        __syncthreads();
        const double* Cin = C0 + c * RK;
        double* Cout = C0 + (c + 1) * RK;
        for (int e = threadIdx.x; e < RK; e += blockDim.x) {
            const int r = e / K, b = e - r * K;
            Cout[e] = m2m(Cin, T[22 + c], r, b, 0.0);
        }
    }
    __syncthreads();
    // the records (mid q1: T[16 + q1]; A: T[20]; chain level c: T[30 + c]), each into
    // this rank's record buffer and every peer part
    const int nrec = 5 + nc;
    for (int f = threadIdx.x; f < nrec * RK; f += blockDim.x) {
        const int j = f / RK, e = f - j * RK;
        const int ri = j < 4 ? T[16 + j] : j == 4 ? T[20] : T[30 + j - 5];
        if (ri < 0) continue;
        const double v = j < 4 ? Mid[f] : C0[f - 4 * RK];
        const int64_t o = (int64_t)ri * RK + e;
        rec[o] = v;
        for (int p = 0; p < nPeer; ++p) buf[PO[p] + o] = v;
    }
}

typedef __attribute__((address_space(1))) unsigned gu32_up;

template <int K>
__global__ void __launch_bounds__(kUpThreads) k_up_tier(
    int taskBase, const int* __restrict__ taskList, int maxTask, const int4* __restrict__ desc, const int* __restrict__ grpFix,
    const int* __restrict__ node, const int4* __restrict__ code, const double4* __restrict__ geom,
    const int2* __restrict__ leafRange, const double* __restrict__ pxT, const double* __restrict__ pyT,
    const double* __restrict__ xin, int64_t ldi, int treeIn, const int* __restrict__ perm,
    const double* __restrict__ sigT, const double* __restrict__ wT, double* __restrict__ fT, double* __restrict__ cT,
    const Params* __restrict__ P, double* __restrict__ mult, const int* __restrict__ rootSlot,
    const double* __restrict__ recv, const int* __restrict__ sendSlot, double* __restrict__ send,
    unsigned* __restrict__ zeroCnt, UpTail tail) {
    extern __shared__ double sm[];
    // the counters of the fused top-of-tree launch that follows (k_top_m2l_hc)
    if (zeroCnt && blockIdx.x == 0 && threadIdx.x <= kMaxTopTiers) zeroCnt[threadIdx.x] = 0u;
    const int task = taskList ? taskList[blockIdx.x] : taskBase + (int)blockIdx.x;
    up_task<K>(task, maxTask, desc, grpFix, node, code, geom, leafRange, pxT, pyT, xin, ldi, treeIn, perm, sigT, wT,
               fT, cT, P, mult, rootSlot, recv, sendSlot, send, sm);
    if (!tail.partOf) return;
    // the partial task's last root (MI355X_MICROARCH.md, inter-workgroup visibility:
    // the last-adder hand-off with a write-through payload, no fences): this block's
    // root multipole (its own plain stores, re-read after the barrier) is copied into
    // the staging slot with sc1 (write-through) stores; every storing wave waits for
    // them, then one lane adds to the partial task's counter; the block whose add
    // completes the count resets the counter for the next apply and runs the partial
    // task, loading the staged roots with sc1 loads.  No block waits for another, so
    // dispatch order does not matter.
    constexpr int RK = kRank * K;
    __shared__ int lastOf;
    const int2 pq = tail.partOf[blockIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the root's plain stores by every wave of this block
    __syncthreads();
    if (pq.x >= 0)
        for (int e = threadIdx.x; e < RK; e += blockDim.x)
            __hip_atomic_store(tail.stage + (size_t)pq.x * RK + e, mult[(size_t)pq.y * RK + e], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        if (pq.x >= 0) {
            const int p = pq.x >> 4;
            const unsigned old = __hip_atomic_fetch_add((gu32_up*)(tail.cnt + p), 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1u == (unsigned)tail.nroots[p]) {
                __hip_atomic_store((gu32_up*)(tail.cnt + p), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                run = p + 1;
            }
        }
        lastOf = run;
    }
    __syncthreads();
    if (lastOf)
        up_partial_task<K>(tail.task + (size_t)(lastOf - 1) * Plan::kUpTaskInts, P, mult, tail.rec, tail.nPeer,
                           tail.peerOff, tail.buf, sm, tail.stage + (size_t)(lastOf - 1) * 16 * RK);
}


// ----------------------------------------------------------------- M2L

// M2L over the V then X lists with the cached merged 16x16 operators
// (bbfmm.h:1051-1065).  HBM-bound stream: one wave per target node, each pair's
// 2 KB operator is read as 64 lanes x 32 contiguous bytes (two dwordx4 loads).
// Blocks are column-major (K[t][s] at s*16 + t): lane l owns column s = l>>2 and
// rows 4(l&3)..4(l&3)+3.  Forward product: per lane partial sums over its column
// for its 4 rows and every base vector, one 16-lane reduction and the mode's mix
// per target.
// Symmetric storage: the target's stored pairs are
// [directed | canonical]; for a canonical pair (n, B) the same block also gives
// B's contribution sgn * K^T mult[n] (4 in-lane FMAs + a DPP quad reduction per
// right-hand side), stored to the receiver's partial slot and gathered by
// k_m2l_gather.  Wave-uniform indexing (readfirstlane) keeps descriptors and
// source ids on the scalar unit; PG blocks (PG x 2 KB) are in flight per wave.
// Entry s of a source multipole (base vectors), every right-hand side.
template <int K>
__device__ __forceinline__ void m2l_source(const double* __restrict__ mult, int srcId, int s, double (&xm)[K]) {
    const double* m = mult + ((size_t)srcId * kRank + s) * K;
#pragma unroll
    for (int b = 0; b < K; ++b) xm[b] = m[b];
}

// Forward contribution of G column-major blocks: lane (s, q) adds K[4q+j][s] x[s].
template <int K, int G>
__device__ __forceinline__ void m2l_forward(const dbl2 (&kb)[G][2], const double (&xm)[G][K], double (&c)[4][K]) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < K; ++i) {
            c[0][i] += kb[g][0].x * xm[g][i];
            c[1][i] += kb[g][0].y * xm[g][i];
            c[2][i] += kb[g][1].x * xm[g][i];
            c[3][i] += kb[g][1].y * xm[g][i];
        }
}

template <int K, int PG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K >= 8 ? 1 : 3))) k_m2l(int ntgt, const int* __restrict__ tgt, const int64_t* __restrict__ ptr,
                                             const int* __restrict__ nDir, const int* __restrict__ canonBase,
                                             const int* __restrict__ outSlot, const int* __restrict__ src,
                                             const ModeArgs* __restrict__ tab, int nterm,
                                             const double* __restrict__ mult, int maxCanon,
                                             double* __restrict__ partial, double* __restrict__ local) {
    // K >= 4: the transposed products wait in LDS (maxCanon x 16 x K doubles per
    // wave) instead of registers
    constexpr bool kLdsY = K >= 4;
    extern __shared__ double ysh[];
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) / kWave));
    const int lane = threadIdx.x & (kWave - 1);
    if (wave >= ntgt) return;
    const int n = tgt[wave];
    const int s = lane >> 2, q = lane & 3;  // column s, rows 4q .. 4q+3
    const int64_t p0 = ptr[wave], p1 = ptr[wave + 1], pd = p0 + nDir[wave];
    const int nC = (int)(p1 - pd);  // canonical pairs, <= maxCanon (host plan)
    const int cSrc = lane < nC ? src[pd + lane] : 0;
    const int cSlot = lane < nC ? outSlot[canonBase[wave] + lane] : 0;
    // transposed products, summed over the terms: registers (lane (s, q) keeps
    // entry s of pair 4g + q, every right-hand side) or, K >= 4, LDS; stored after
    // the stream (on CDNA vmcnt also counts stores: stores inside the loop stall it)
    constexpr int kGroups = kLdsY ? 1 : (kMaxCanon + 3) / 4;
    double y[kGroups][K];
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
#pragma unroll
        for (int i = 0; i < K; ++i) y[g][i] = 0.0;
    double* yl = ysh + (size_t)(threadIdx.x / kWave) * maxCanon * kRank * K;
    if constexpr (kLdsY) {
        for (int e = lane; e < nC * kRank * K; e += kWave) yl[e] = 0.0;
    }
    // this lane's outputs: row t = s, right-hand sides i = q and q + 4
    double lo[2] = {0.0, 0.0};
#pragma unroll 1
    for (int term = 0; term < nterm; ++term) {
        const ModeArgs& md = tab[term];
        const double* __restrict__ Kop = md.Km2l;
        double c[4][K];  // forward: rows 4q+j, this lane's column, each base vector
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < K; ++i) c[j][i] = 0.0;
        // ---- directed pairs, PG blocks in flight
        for (int64_t cb = p0; cb < pd; cb += kWave) {
            const int cnt = (int)min<int64_t>(kWave, pd - cb);
            const int mySrc = lane < cnt ? src[cb + lane] : 0;
            for (int j = 0; j < cnt; j += PG) {
                dbl2 kb[PG][2];
                double xm[PG][K];
#pragma unroll
                for (int g = 0; g < PG; ++g) load_block(Kop, cb + j + g, lane, j + g < cnt, kb[g][0], kb[g][1]);
#pragma unroll
                for (int g = 0; g < PG; ++g)  // a skipped block's source is a valid clamp; its block is zero
                    m2l_source<K>(mult, __builtin_amdgcn_readlane(mySrc, min(j + g, cnt - 1)), s, xm[g]);
                m2l_forward<K, PG>(kb, xm, c);
            }
        }
        // ---- canonical pairs: both products from one read of the block
        if (nC > 0) {
            double mn[4][K];  // the target's multipole, mixed, rows 4q+j, times sgn
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double base[K];
#pragma unroll
                for (int b = 0; b < K; ++b) base[b] = mult[((size_t)n * kRank + 4 * q + j) * K + b];
                mix_apply_t<K>(md, base, mn[j]);
#pragma unroll
                for (int i = 0; i < K; ++i) mn[j][i] *= md.sgn;
            }
            // one group: CG blocks in flight (4; 2 with LDS staging, for registers),
            // forward + transposed products; lane q adds pair CG g + q
            constexpr int CG = kLdsY ? 2 : 4;
            auto group = [&](int g, double (&yg)[K]) {
                const int j = CG * g;
                dbl2 kb[CG][2];
                double xm[CG][K];
#pragma unroll
                for (int u = 0; u < CG; ++u) load_block(Kop, pd + j + u, lane, j + u < nC, kb[u][0], kb[u][1]);
#pragma unroll
                for (int u = 0; u < CG; ++u)
                    m2l_source<K>(mult, __builtin_amdgcn_readlane(cSrc, min(j + u, nC - 1)), s, xm[u]);
                m2l_forward<K, CG>(kb, xm, c);
#pragma unroll
                for (int u = 0; u < CG; ++u)
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const double v = quad_sum(kb[u][0].x * mn[0][i] + kb[u][0].y * mn[1][i] +
                                                  kb[u][1].x * mn[2][i] + kb[u][1].y * mn[3][i]);
                        if (u == q) yg[i] += v;
                    }
            };
            if constexpr (kLdsY) {
                for (int g = 0; CG * g < nC; ++g) {
                    double yt[K];
#pragma unroll
                    for (int i = 0; i < K; ++i) yt[i] = 0.0;
                    group(g, yt);
                    if (q < CG && CG * g + q < nC)
#pragma unroll
                        for (int i = 0; i < K; ++i) yl[((size_t)(CG * g + q) * kRank + s) * K + i] += yt[i];
                }
            } else {
#pragma unroll
                for (int g = 0; g < kGroups; ++g)
                    if (4 * g < nC) group(g, y[g]);
            }
        }
        // ---- sum the forward partials over the 16 columns (lane bits 2..5); then
        // row t = 4q' + j is entry j of the lanes with q == q' (e.g. lane 4t + (t>>2));
        // the sums are over base multipoles: the term's mix is applied here, per row
#pragma unroll
        for (int off = 4; off < kWave; off <<= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) c[j][i] += __shfl_xor(c[j][i], off);
        const int jr = s & 3, srcLane = 4 * s + (s >> 2);
        double v[K];
#pragma unroll
        for (int b = 0; b < K; ++b) {
            const double sel = jr == 0 ? c[0][b] : jr == 1 ? c[1][b] : jr == 2 ? c[2][b] : c[3][b];
            v[b] = __shfl(sel, srcLane);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            if ((i & 3) != q) continue;
            double w = 0.0;
#pragma unroll
            for (int b = 0; b < K; ++b) w += md.mix[i][b] * v[b];
            lo[i >> 2] += w;
        }
    }
    double* dst = local + ((size_t)n * kRank + s) * K;
#pragma unroll
    for (int i = 0; i < K; ++i)
        if ((i & 3) == q) dst[i] = lo[i >> 2];
    if (nC == 0) return;
    if constexpr (kLdsY) {
        // partial slots: pair p's 16 K doubles are contiguous in LDS and in its
        // slot; slot ids shuffled with every lane active
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        constexpr int PE = kRank * K;
        for (int e0 = 0; e0 < nC * PE; e0 += kWave) {
            const int e = e0 + lane;
            const int pr = min(e / PE, nC - 1);
            const int slot = __shfl(cSlot, pr);
            if (e < nC * PE) partial[(size_t)slot * PE + (e - pr * PE)] = yl[e];
        }
    } else {
        // partial slots: lane (s, q) stores entry s of pair 4g + q (K contiguous
        // doubles; 16 K contiguous per pair); slot ids shuffled with every lane active
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
            if (4 * g < nC) {
                const int jj = 4 * g + q;
                const int slot = __shfl(cSlot, jj);
                if (jj < nC) {
                    double* dstp = partial + ((size_t)slot * kRank + s) * K;
#pragma unroll
                    for (int i = 0; i < K; ++i) dstp[i] = y[g][i];
                }
            }
        }
    }
}

// local[B] += the transposed canonical-pair products addressed to B: one
// contiguous slot range per target, summed in a fixed order (deterministic).
// One thread per (target, entry, right-hand side); 8 loads in flight per thread.
template <int K>
__global__ void __launch_bounds__(256) k_m2l_gather(int ntgt, const int* __restrict__ tgt,
                                                    const int* __restrict__ inPtr, const double* __restrict__ partial,
                                                    double* __restrict__ local) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t w = gid / (kRank * K);
    const int e = (int)(gid - w * (kRank * K));  // entry * K + rhs
    if (w >= ntgt) return;
    const int j0 = inPtr[w], j1 = inPtr[w + 1];
    if (j0 == j1) return;
    const double* pp = partial + (size_t)j0 * kRank * K + e;
    const int n = j1 - j0;
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int j = 0;
    for (; j + 7 < n; j += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += __builtin_nontemporal_load(pp + (size_t)(j + u) * kRank * K);
    }
#pragma unroll
    for (int u = 0; u < 7; ++u)
        if (j + u < n) a[u] += __builtin_nontemporal_load(pp + (size_t)(j + u) * kRank * K);
    local[(size_t)tgt[w] * kRank * K + e] += ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// ----------------------------------------------------------------- near field

// Sum over the lpc lanes of a column group (lpc a power of two, wave-uniform):
// DPP quad exchanges for the first two steps, swizzles above.
__device__ __forceinline__ double group_sum(double v, int lpc) {
    if (lpc >= 2) v += dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
    if (lpc >= 4) v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
    for (int off = 4; off < lpc; off <<= 1) v += __shfl_xor(v, off);
    return v;
}

// U/W near field with symmetric U storage, one target leaf per wave
// (bbfmm.h:1081-1099, 1111-1113).  All per-leaf indexing comes from host-built descriptors loaded lane-parallel:
//   leafInfo[li] = (node, begin, count, S), nearPts = the S source tree positions.
// The S base source charges are staged in LDS ([S][K], unmixed).  The block is
// column-major nT4 x S (rows padded to a multiple of 4): lane (row quad rq,
// column phase) reads 32 B = rows 4rq..4rq+3 of one column, two to four columns
// in flight.  Forward: per-lane sums over its columns of the base charges, one
// cross-lane reduction per leaf, then the mode's mix applied to the nT outputs
// (linear: mixing the sums equals summing the mixed charges, at nT instead of S
// mixes).  Canonical U pairs (host: both leaves <= 128 points):
// the same column read also gives the other leaf's transposed product
// sgn * sum_t K[t][s] f_mix[t], reduced over the column's lanes (DPP), staged in
// LDS over the consumed charges and stored after the stream.  accum: add to out
// and to the partials (later modes of a block apply) instead of storing.
template <int K>
__global__ void __launch_bounds__(256) k_near_sym(int nl, const int4* __restrict__ leafInfo,
                                              const int64_t* __restrict__ nearPtsPtr, const int* __restrict__ nearPts,
                                              const int64_t* __restrict__ nearKOff, const int2* __restrict__ nearSym,
                                              const double* __restrict__ Kop, const double* __restrict__ fT,
                                              MixK<K> mix, const int* __restrict__ operm, int64_t obase, int64_t ldo,
                                              int maxS, int flags, double sgn, double scale, int accum,
                                              double* __restrict__ partial, double* __restrict__ out) {
    extern __shared__ double sh[];
    const int wv = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    const int li = blockIdx.x * (blockDim.x / kWave) + wv;
    const bool active = li < nl;
    double* fs = sh + (size_t)wv * maxS * K;
    int4 info = make_int4(0, 0, 0, 0);
    int64_t koff = 0;
    if (active) {
        info = leafInfo[li];
        const int64_t pb = nearPtsPtr[li];
        koff = nearKOff[li];
        // stage the S x K base charges: lane-contiguous (source, rhs) entries (the
        // points of one source leaf are contiguous in tree order), 4 in flight
        const int SK = info.w * K;
        for (int e0 = 0; e0 < SK; e0 += 4 * kWave) {
            double fv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = e0 + u * kWave + lane;
                fv[u] = e < SK ? fT[(size_t)nearPts[pb + e / K] * kStride<K> + e % K] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = e0 + u * kWave + lane;
                if (e < SK) fs[e] = fv[u];
            }
        }
    }
    __syncthreads();
    if (!active) return;
    const int nT = info.z, S = info.w;
    const int2 sym = nearSym[li];  // (directed source points Sdir, partial base)
    const int Sdir = sym.x;
    const int64_t tb = info.y;
    const int nq = (nT + 3) >> 2;  // row quads
    const int cstr = 2 * nq;       // column stride in 16-B units
    int lpc = 1;                   // lanes per column
    while (lpc < nq && lpc < kWave) lpc <<= 1;
    const int cps = kWave / lpc;
    const int cph = lane / lpc;
    const bool nearOn = flags & kStageNear;
    for (int rc = 0; rc < nq; rc += kWave) {  // > 64 row quads: leaves over 256 points (directed only)
        const int rq = rc + (lane & (lpc - 1));
        const bool rowOk = rq < nq;
        const dbl2* kc = reinterpret_cast<const dbl2*>(Kop + koff) + 2 * rq;
        double a[4][K];  // forward: rows 4rq+j, base charges
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < K; ++b) a[j][b] = 0.0;
        if (nearOn && S > Sdir) {
            double fa[4][K];  // this leaf's mixed charges at rows 4rq+j, times sgn
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double bv[K];
                const bool ok = rowOk && 4 * rq + j < nT;
#pragma unroll
                for (int b = 0; b < K; ++b) bv[b] = ok ? fT[(size_t)(tb + 4 * rq + j) * kStride<K> + b] : 0.0;
                mix_apply(mix, bv, fa[j]);
#pragma unroll
                for (int i = 0; i < K; ++i) fa[j][i] *= sgn;
            }
            const int ncol = S - Sdir;
            for (int i0 = 0; i0 < ncol; i0 += 2 * cps) {  // 2 columns per lane in flight
                dbl2 kk[2][2];
                bool ok[2];
                int sc[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int c = i0 + u * cps + cph;
                    ok[u] = c < ncol && rowOk;
                    sc[u] = Sdir + min(c, ncol - 1);
                    const dbl2* p = kc + (size_t)sc[u] * cstr;
                    kk[u][0] = ok[u] ? __builtin_nontemporal_load(p) : dbl2{0.0, 0.0};
                    kk[u][1] = ok[u] ? __builtin_nontemporal_load(p + 1) : dbl2{0.0, 0.0};
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    double* fc = fs + (size_t)sc[u] * K;
                    const double k4[4] = {kk[u][0].x, kk[u][0].y, kk[u][1].x, kk[u][1].y};
#pragma unroll
                    for (int b = 0; b < K; ++b) {
                        const double fv = fc[b];
#pragma unroll
                        for (int j = 0; j < 4; ++j) a[j][b] += k4[j] * fv;
                    }
                    double y[K];
#pragma unroll
                    for (int i = 0; i < K; ++i)
                        y[i] = group_sum(k4[0] * fa[0][i] + k4[1] * fa[1][i] + k4[2] * fa[2][i] + k4[3] * fa[3][i],
                                         lpc);
                    // column sc's charges are consumed (every lane of the group has
                    // read them above): its LDS words now hold the product, stored
                    // after the stream (vmcnt also counts stores)
                    if (ok[u] && (lane & (lpc - 1)) == 0)
#pragma unroll
                        for (int i = 0; i < K; ++i) fc[i] = y[i];
                }
            }
        }
        if (nearOn && rowOk) {
            int sc = cph;
            for (; sc + 3 * cps < Sdir; sc += 4 * cps) {
                dbl2 kk[4][2];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const dbl2* p = kc + (size_t)(sc + u * cps) * cstr;
                    kk[u][0] = __builtin_nontemporal_load(p);
                    kk[u][1] = __builtin_nontemporal_load(p + 1);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double* fc = fs + (size_t)(sc + u * cps) * K;
#pragma unroll
                    for (int b = 0; b < K; ++b) {
                        const double fv = fc[b];
                        a[0][b] += kk[u][0].x * fv;
                        a[1][b] += kk[u][0].y * fv;
                        a[2][b] += kk[u][1].x * fv;
                        a[3][b] += kk[u][1].y * fv;
                    }
                }
            }
            for (; sc < Sdir; sc += cps) {
                const dbl2* p = kc + (size_t)sc * cstr;
                const dbl2 k0 = __builtin_nontemporal_load(p), k1 = __builtin_nontemporal_load(p + 1);
                const double* fc = fs + (size_t)sc * K;
#pragma unroll
                for (int b = 0; b < K; ++b) {
                    const double fv = fc[b];
                    a[0][b] += k0.x * fv;
                    a[1][b] += k0.y * fv;
                    a[2][b] += k1.x * fv;
                    a[3][b] += k1.y * fv;
                }
            }
        }
        // sum over the column phases (lane bits above the column group)
        for (int off = lpc; off < kWave; off <<= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int b = 0; b < K; ++b) a[j][b] += __shfl_xor(a[j][b], off);
        if (cph == 0 && rowOk) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = 4 * rq + j;
                if (t >= nT) break;
                const int64_t o = out_index(operm, obase, tb + t);
                double v[K];
                mix_apply(mix, a[j], v);
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    double* dst = out + (size_t)i * ldo + o;
                    *dst = accum ? *dst + scale * v[i] : scale * v[i];
                }
            }
        }
    }
    if (nearOn && S > Sdir) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int nv = (S - Sdir) * K;
        double* dst = partial + (size_t)sym.y * K;
        const double* src = fs + (size_t)Sdir * K;
        for (int i = lane; i < nv; i += kWave) dst[i] = accum ? dst[i] + src[i] : src[i];
    }
}

// U/W near field, directed storage (every U/W block stored for its target; the
// layout of block handles), all mode terms in one launch: G lanes
// per target leaf (G = 16 when every leaf has <= 16 points, 4 leaves per wave;
// else 64).  The block is column-major nT4 x S (rows padded to a multiple of 4);
// lane (row quad rq, column phase) reads 32 B = rows 4rq..4rq+3 of a column and
// the column's K base charges straight from fT (L1/L2: the lanes of a column
// share the line), U columns in flight per lane.  Per term: forward sums per lane
// over its columns, one reduction over the column phases (DPP row rotations for
// G = 16), the term's mix at the outputs; out is written once.  No LDS, no partials.
template <int K, int G, int U>
__global__ void __launch_bounds__(256) k_near(int nl, const int4* __restrict__ leafInfo,
                                              const int64_t* __restrict__ nearPtsPtr, const int* __restrict__ nearPts,
                                              const int64_t* __restrict__ nearKOff, const ModeArgs* __restrict__ tab,
                                              int nterm, const double* __restrict__ fT,
                                              const int* __restrict__ operm, int64_t obase, int64_t ldo, int flags,
                                              double scale, int accum, double* __restrict__ out) {
    static_assert(G == 16 || G == 64, "leaf group of 16 or 64 lanes");
    constexpr int KS = kStride<K>;
    const int gl = threadIdx.x & (G - 1);
    const int li = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G);
    const bool active = li < nl;
    int4 info = make_int4(0, 0, 0, 0);
    int64_t pb = 0, koff = 0;
    if (active) {
        info = leafInfo[li];
        pb = nearPtsPtr[li];
        koff = nearKOff[li];
    }
    const int nT = info.z, S = (flags & kStageNear) ? info.w : 0;
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
        // outputs of this lane summed over the terms: G = 16 row 4rq + cph; G = 64
        // rows 4rq + j on column phase 0
        constexpr int NR = (G == 16) ? 1 : 4;
        double o[NR][K];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int b = 0; b < K; ++b) o[r][b] = 0.0;
        for (int term = 0; term < nterm; ++term) {
            const ModeArgs& md = tab[term];
            const dbl2* kc = reinterpret_cast<const dbl2*>(md.Knear + koff) + 2 * rq;
            double a[4][K];  // rows 4rq+j, base charges
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int b = 0; b < K; ++b) a[j][b] = 0.0;
            if (rowOk) {
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
                    double f[U][K];
#pragma unroll
                    for (int u = 0; u < U; ++u) load_charges<K>(fT + (size_t)ix[u] * KS, f[u]);
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int b = 0; b < K; ++b) {
                            a[0][b] += kk[u][0].x * f[u][b];
                            a[1][b] += kk[u][0].y * f[u][b];
                            a[2][b] += kk[u][1].x * f[u][b];
                            a[3][b] += kk[u][1].y * f[u][b];
                        }
                }
            }
            // sum over the column phases: G = 16 -> lanes 4 and 8 apart in a 16-lane row
            if constexpr (G == 16) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int b = 0; b < K; ++b) {
                        double v = a[j][b];
                        v += dpp_f64<0x124>(v);  // row_ror:4
                        v += dpp_f64<0x128>(v);  // row_ror:8
                        a[j][b] = v;
                    }
                // this lane's row 4rq + cph, mixed
                double r[K];
#pragma unroll
                for (int b = 0; b < K; ++b) r[b] = cph == 0 ? a[0][b] : cph == 1 ? a[1][b] : cph == 2 ? a[2][b] : a[3][b];
                double v[K];
                mix_apply_t<K>(md, r, v);
#pragma unroll
                for (int i = 0; i < K; ++i) o[0][i] += v[i];
            } else {
                for (int off = lpc; off < kWave; off <<= 1)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int b = 0; b < K; ++b) a[j][b] += __shfl_xor(a[j][b], off);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    double v[K];
                    mix_apply_t<K>(md, a[j], v);
#pragma unroll
                    for (int i = 0; i < K; ++i) o[NR == 4 ? j : 0][i] += v[i];
                }
            }
        }
        if (rowOk) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = 4 * rq + j;
                const bool mine = (G == 16) ? (cph == j) : (cph == 0);
                if (!mine || t >= nT) continue;
                const int64_t oi = out_index(operm, obase, tb + t);
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const double v = scale * o[NR == 4 ? j : 0][i];
                    double* dst = out + (size_t)i * ldo + oi;
                    *dst = accum ? *dst + v : v;
                }
            }
        }
        if constexpr (G == 16) break;
    }
}

// ----------------------------------------------------------------- down pass

// Down pass (bbfmm.h:1066-1106) over the owned subtree tasks, after k_m2l,
// k_m2l_gather and k_near.  Every task rebuilds its root's parent total from the
// ancestors' locals (L2L chain from level 1), so all tasks are independent.  Per
// node: total = local (its M2L, transposed partials included) + L2L of the
// parent's total (bbfmm.h:1070-1071).  Then per owned leaf point: L2P
// (bbfmm.h:1104) + the gathered transposed U-pair products, added to out.
// dn = (node, parent code: LDS slot, -1 none/zero, -2 the task root; child slot, 0).
// Phase 0 issues every independent global load of the task at once (locals of
// all nodes and chain ancestors, leaf boxes, near partial offsets) into LDS.
#ifdef ANISO_DOWN_TRACE  // development variant: per-task phase timestamps of the down pass
__device__ long long g_downTrace[16384 * 6];
__device__ __forceinline__ void down_mark(int f) {
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 16384) {
        g_downTrace[blockIdx.x * 6 + f] = (long long)__builtin_amdgcn_s_memrealtime();
        if (f == 0) g_downTrace[blockIdx.x * 6 + 5] = (long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    }
}
#define DOWN_MARK(f) down_mark(f)
#else
#define DOWN_MARK(f)
#endif

template <int K>
__global__ void __launch_bounds__(kTierThreads) k_down_tier(
    int maxTask, int maxLeaves, const int4* __restrict__ desc, const int* __restrict__ grpFix,
    const int4* __restrict__ dn, const double* __restrict__ local, const Params* __restrict__ P,
    const int* __restrict__ leafSlot, const int* __restrict__ leafBegin, const int2* __restrict__ leafNear,
    const double4* __restrict__ leafGeom, const double* __restrict__ pxT, const double* __restrict__ pyT,
    const int* __restrict__ operm, int64_t obase, int64_t ldo, const int* __restrict__ nearOff, int maxNear,
    const double* __restrict__ nearPart, const int2* __restrict__ chain, int maxChain, int flags, double scale,
    double* __restrict__ out, const double* __restrict__ xsub, int64_t ldx, const double* __restrict__ hpart,
    const int* __restrict__ chainFold) {
    constexpr int RK = kRank * K;
    extern __shared__ double sm[];
    int4* DN = reinterpret_cast<int4*>(sm);                // maxTask node records
    double* Rl = reinterpret_cast<double*>(DN + maxTask);  // 4 x 256 transfer matrices
    double* T = Rl + 4 * kRank * kRank;                    // maxTask x 16 x K totals
    double* PT = T + (size_t)maxTask * RK;                 // 16 x K: the task root's parent total
    double* CH = PT + RK;                                  // maxChain x 16 x K: the ancestors' locals
    double* G = CH + (size_t)maxChain * RK;                // maxLeaves x 4: leaf cx, cy, 1/rx, 1/ry
    int* LB = reinterpret_cast<int*>(G + (size_t)maxLeaves * 4);  // maxLeaves + 1: leaf begins
    int* LS = LB + maxLeaves + 1;                          // maxLeaves: leaf slot in the task
    int* NB = LS + maxLeaves;                              // maxLeaves: first of the leaf's near offsets in NO
    int* NC = NB + maxLeaves;                              // maxLeaves: their count
    int* NO = NC + maxLeaves;                              // maxNear: partial offsets addressed to this task
    int2* CN = reinterpret_cast<int2*>(NO + maxNear + ((maxNear + 1) & 1));  // maxChain: (ancestor, child index), 8-B aligned
    int* CF = reinterpret_cast<int*>(CN + maxChain);       // maxChain: the ancestors' halo partials (packed)
    const int task = blockIdx.x;
    DOWN_MARK(0);
    // task record: (first node, nodes, first leaf entry, leaves), (owned points begin,
    // end, first chain entry, chain length), (first near offset, count, levels, 0)
    const int4 d0 = desc[3 * task], d1 = desc[3 * task + 1], d2 = desc[3 * task + 2];
    const int n0 = d0.x, nt = d0.y, l0 = d0.z, nl = d0.w;
    const int2 pr = make_int2(d1.x, d1.y);
    const int c0 = d1.z, nc = d1.w;
    const int npts = pr.y - pr.x, ngrp = d2.z;
    const int* gs = grpFix + (size_t)task * (kTaskLevels + 1);
    const bool far = flags & kStageFar;
    // ---- phase 0: the task's records, then (one more round) the locals they address --
    // every load of a round independent, none behind another global load
    if (far) {
        for (int i = threadIdx.x; i < 4 * kRank * kRank; i += blockDim.x) Rl[i] = (&P->R[0][0])[i];
        for (int k = threadIdx.x; k < nt; k += blockDim.x) DN[k] = dn[n0 + k];
        for (int k = threadIdx.x; k < nc; k += blockDim.x) {
            CN[k] = chain[c0 + k];
            CF[k] = hpart && chainFold ? chainFold[c0 + k] : 0;  // no chain records: no chain partials
        }
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
    if (far) {
        // a node's local = its cluster's store + the halo partials other clusters left
        // for it (the halo form of the cluster M2L: packed (first << 3) | count, one
        // receiver-contiguous range), all loads of one round
        // (every load of an entry issued before its sum: the partials' count is a
        // runtime value, and a loop over it waited on each load in turn)
        auto total = [&](int n, int fold, int e) {
            const int cnt = fold & 7;  // fold = 0 when there are no partials (hpart may be null)
            double v = local[(size_t)n * RK + e];
            if (cnt > 0) {
                const double* hp = hpart + (size_t)(fold >> 3) * RK + e;
                double p[7];
#pragma unroll
                for (int j = 0; j < 7; ++j) p[j] = hp[(size_t)min(j, cnt - 1) * RK];  // clamped: a valid slot
#pragma unroll
                for (int j = 0; j < 7; ++j)
                    if (j < cnt) v += p[j];
            }
            return v;
        };
        for (int it = threadIdx.x; it < nt * RK; it += blockDim.x) {
            const int4 d = DN[it / RK];
            T[it] = total(d.x, hpart ? d.w : 0, it % RK);
        }
        for (int it = threadIdx.x; it < nc * RK; it += blockDim.x) CH[it] = total(CN[it / RK].x, CF[it / RK], it % RK);
        __syncthreads();
    }
    DOWN_MARK(1);
    // ---- phase 1: the root's parent total by the L2L chain from level 1
    // (bbfmm.h:1070-1071 along the ancestors), then the task's levels
    if (far) {
        if constexpr (RK <= kWave) {  // one wave, lane (r, i) = r K + i; no barrier per step
            if (threadIdx.x < kWave) {
                const int r = threadIdx.x / K, i = threadIdx.x - (threadIdx.x / K) * K;
                double v = (nc > 0 && threadIdx.x < RK) ? CH[threadIdx.x] : 0.0;
                for (int jc = 1; jc < nc; ++jc) {
                    const double* R = Rl + CN[jc].y * kRank * kRank;
                    double a = threadIdx.x < RK ? CH[jc * RK + threadIdx.x] : 0.0;
#pragma unroll
                    for (int c = 0; c < kRank; ++c) a += R[(r & 15) + c * kRank] * __shfl(v, c * K + i);
                    v = a;
                }
                if (threadIdx.x < RK) PT[threadIdx.x] = v;
            }
        } else {  // PT holds the running total; one thread per (entry, rhs), barriers per step
            for (int it = threadIdx.x; it < RK; it += blockDim.x) PT[it] = nc > 0 ? CH[it] : 0.0;
            __syncthreads();
            for (int jc = 1; jc < nc; ++jc) {
                const double* R = Rl + CN[jc].y * kRank * kRank;
                const int r = threadIdx.x / K, i = threadIdx.x - (threadIdx.x / K) * K;
                double a = 0.0;
                if (threadIdx.x < RK) {
                    a = CH[jc * RK + threadIdx.x];
#pragma unroll
                    for (int c = 0; c < kRank; ++c) a += R[r + c * kRank] * PT[c * K + i];
                }
                __syncthreads();
                if (threadIdx.x < RK) PT[threadIdx.x] = a;
                __syncthreads();
            }
        }
        __syncthreads();
        DOWN_MARK(2);
        for (int g = 0; g < ngrp; ++g) {
            const int s0 = gs[g], s1 = gs[g + 1];
            for (int it = threadIdx.x; it < (s1 - s0) * kRank; it += blockDim.x) {
                const int k = s0 + (it >> 4), r = it & (kRank - 1);
                const int4 d = DN[k];
                if (d.y == -1) continue;
                const double* pt = d.y >= 0 ? T + (size_t)d.y * RK : PT;  // -2: the task root
                const double* R = Rl + d.z * kRank * kRank;
                double l2l[K];
#pragma unroll
                for (int i = 0; i < K; ++i) l2l[i] = 0.0;
#pragma unroll
                for (int c = 0; c < kRank; ++c) {
                    const double rc = R[r + c * kRank];
#pragma unroll
                    for (int i = 0; i < K; ++i) l2l[i] += rc * pt[c * K + i];
                }
#pragma unroll
                for (int i = 0; i < K; ++i) T[((size_t)k * kRank + r) * K + i] += l2l[i];
            }
            __syncthreads();
        }
    }
    DOWN_MARK(3);
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
        double v[K];
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = 0.0;
        if ((flags & kStageNear) && nearPart) {  // nullptr: this apply's near field left no partials
            const int* no = NO + NB[lo];
            for (int j = 0; j < NC[lo]; ++j) {
                const double* pp = nearPart + ((size_t)no[j] + t) * K;
#pragma unroll
                for (int i = 0; i < K; ++i) v[i] += pp[i];
            }
        }
        if (far) {
            const double x = pxT[kpos], y = pyT[kpos];
            double Sx[kNP], Sy[kNP];
            cheb_weights(P, (x - G[4 * lo]) * G[4 * lo + 2], Sx);
            cheb_weights(P, (y - G[4 * lo + 1]) * G[4 * lo + 3], Sy);
            const double* L = T + (size_t)LS[lo] * RK;
            double l2p[K];
#pragma unroll
            for (int i = 0; i < K; ++i) l2p[i] = 0.0;
#pragma unroll
            for (int j = 0; j < kNP; ++j)
#pragma unroll
                for (int ii = 0; ii < kNP; ++ii) {
                    const double w = Sx[ii] * Sy[j];
#pragma unroll
                    for (int i = 0; i < K; ++i) l2p[i] += w * L[(j * kNP + ii) * K + i];
                }
#pragma unroll
            for (int i = 0; i < K; ++i) v[i] += l2p[i];
        }
        const int64_t o = out_index(operm, obase, kpos);
        if (xsub) {  // aniso.m's x - mforward(x) fused into the last writer (aniso.m:155)
#pragma unroll
            for (int i = 0; i < K; ++i)
                out[(size_t)i * ldo + o] = xsub[(size_t)i * ldx + o] - (out[(size_t)i * ldo + o] + scale * v[i]);
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) out[(size_t)i * ldo + o] += scale * v[i];
        }
    }
    DOWN_MARK(4);
}

#ifdef ANISO_DOWN_TRACE
extern "C" __attribute__((visibility("default"))) int aniso_debug_down_trace(long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_downTrace), (size_t)n * 6 * sizeof(long long)) == hipSuccess ? 0 : 1;
}
#endif

// ----------------------------------------------------------------- corrections

// Corrections (nearRemoval + refineAddOnFast + singularAddFast,
// KernelFactory.cpp:445-478, 662-709, 828-860) as a 3x3-square stencil with
// translation-invariant d2 x 9 x d2 weights, plus the singular term from Legendre
// coefficients of the target's own square (O(d^4) moments).  Both are linear in
// the charges and their per-mode tables are small, so every mode term of a batched
// apply is folded into ONE table on the host with the terms' mixes
// (Operator::corrTable): Wc[tq][q9][c][i][b] = sum_t mix_t[i][b] C_t[tq][q9][c],
// Wm[tq][i][b][a][bb] = sum_t mix_t[i][b] mu_t[tq][a][bb].  One pass per point:
// each neighbour charge is loaded once (d = 1: every weight is wave-uniform).
// Every contribution carries the final 1/(2 pi) (AnisoWrapper.cpp:129-130): the
// near field stores its scaled sum, k_corr and k_down_tier add theirs.
template <int D, int K>
__global__ void __launch_bounds__(256) k_corr(int64_t b, int64_t e, const int* __restrict__ perm,
                                              const int* __restrict__ iperm, const double* __restrict__ cT,
                                              const double* __restrict__ fT, const double* __restrict__ Wc,
                                              const double* __restrict__ Wm, const Params* __restrict__ P, int flags,
                                              double scale, bool treeOut, int64_t ldo, double* __restrict__ out) {
    constexpr int KS = kStride<K>;
    int64_t k = b + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= e) return;
    const int t = perm[k];
    double acc[K];
    corr_point<D, K>(t, P, iperm, [&](int64_t p, int r) { return cT[(size_t)p * KS + r]; }, Wc, Wm, flags,
                     [&](int, int sq2, int c, double (&f)[K]) {
                         load_charges<K>(fT + (size_t)iperm[(size_t)sq2 * (D * D) + c] * KS, f);
                     },
                     acc);
    const int64_t o = treeOut ? k - b : (int64_t)t;
#pragma unroll
    for (int r = 0; r < K; ++r) out[(size_t)r * ldo + o] += acc[r] * scale;
}

// ----------------------------------------------------------------- launchers

template <int K>
static MixK<K> make_mix(const double* m) {  // m: K x K row-major host array
    MixK<K> x;
    for (int i = 0; i < K; ++i)
        for (int b = 0; b < K; ++b) x.c[i][b] = m[i * K + b];
    return x;
}

#define ANISO_DISPATCH_K(k, CALL)                               \
    switch (k) {                                                \
        case 1: { constexpr int KK = 1; CALL; } break;          \
        case 2: { constexpr int KK = 2; CALL; } break;          \
        case 4: { constexpr int KK = 4; CALL; } break;          \
        case 5: { constexpr int KK = 5; CALL; } break;          \
        case 8: { constexpr int KK = 8; CALL; } break;          \
        default: throw std::invalid_argument("unsupported right-hand-side count " + std::to_string(k)); \
    }

bool rhs_supported(int k) { return k == 1 || k == 2 || k == 4 || k == 5 || k == 8; }
int rhs_stride(int k) { return (k == 1 || k % 2 == 0) ? k : k + 1; }
int rhs_padded(int k) {
    for (int c : {1, 2, 4, 5, 8})
        if (k <= c) return c;
    return -1;
}

void launch_prepare(int K, int64_t N, const double* xin, int64_t ldi, int treeIn, const int* perm,
                    const double* sigT, const double* wT, double* fT, double* cT, hipStream_t s) {
    if (N <= 0) return;
    ANISO_DISPATCH_K(K, (k_prepare<KK><<<blocks_for(N, 256), 256, 0, s>>>(N, xin, ldi, treeIn, perm, sigT, wT, fT, cT)));
    HIP_LAUNCH_CHECK();
}

void launch_sub_slice(int64_t n, int nrhs, const double* x, int64_t ldx, const double* a, int64_t lda, double* y,
                      int64_t ldy, hipStream_t s) {
    if (n <= 0 || nrhs <= 0) return;
    k_sub_slice<<<blocks_for(n * nrhs, 256), 256, 0, s>>>(n, nrhs, x, ldx, a, lda, y, ldy);
    HIP_LAUNCH_CHECK();
}

size_t up_tier_lds(int maxTask, int K) {
    return (size_t)(4 * kRank * kRank + maxTask * (kRank * K + 4)) * sizeof(double) +
           (size_t)7 * maxTask * sizeof(int) + (size_t)maxTask * sizeof(int4);  // LB, LC, ND, RS (4 per node)
}

size_t down_tier_lds(int maxTask, int maxLeaves, int maxNear, int maxChain, int K) {
    return (size_t)(4 * kRank * kRank + (maxTask + 1 + maxChain) * kRank * K + 4 * maxLeaves) * sizeof(double) +
           (size_t)(4 * maxLeaves + 4 + maxNear) * sizeof(int) + (size_t)maxTask * sizeof(int4) +
           (size_t)maxChain * (sizeof(int2) + sizeof(int));
}

void launch_up_tier(int K, int ntask, int taskBase, const int* taskList, int maxTask, const int4* desc,
                    const int* grpFix, const int* node, const int4* code, const double4* geom, const int2* leafRange,
                    const double* pxT, const double* pyT, const double* xin, int64_t ldi, int treeIn, const int* perm,
                    const double* sigT, const double* wT, double* fT, double* cT, const Params* P, double* mult,
                    const int* rootSlot, const double* recv, const int* sendSlot, double* send, hipStream_t s,
                    unsigned* zeroCnt, const UpTail* tail) {
    if (ntask <= 0) {
        if (zeroCnt) {
            const hipError_t e = hipMemsetAsync(zeroCnt, 0, (kMaxTopTiers + 1) * sizeof(unsigned), s);
            if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
        }
        return;
    }
    const UpTail tl = tail ? *tail : UpTail{};
    ANISO_DISPATCH_K(K, ({
        const size_t shm = std::max(up_tier_lds(maxTask, KK),
                                    tl.partOf ? (size_t)up_partial_lds<KK>() * sizeof(double) : (size_t)0);
        k_up_tier<KK><<<ntask, kUpThreads, shm, s>>>(taskBase, taskList, maxTask, desc, grpFix, node, code, geom,
                                                     leafRange, pxT, pyT, xin, ldi, treeIn, perm, sigT, wT, fT, cT, P,
                                                     mult, rootSlot, recv, sendSlot, send, zeroCnt, tl);
    }));
    HIP_LAUNCH_CHECK();
}

// Tier-0 root records of a sharded apply without upper tiers: one thread per
// double, records of 16 K contiguous doubles ([node][16][K] multipole layout).
__global__ void k_roots_unpack(int64_t total, int rec, const int* __restrict__ nodes, const double* __restrict__ recv,
                               double* __restrict__ mult) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t j = i / rec, e = i - j * rec;
    const int n = nodes[j];
    if (n >= 0) mult[(int64_t)n * rec + e] = recv[i];
}

void launch_roots_unpack(int K, int nslots, const int* nodes, const double* recv, double* mult, hipStream_t s) {
    const int64_t total = (int64_t)nslots * kRank * K;
    if (total <= 0) return;
    k_roots_unpack<<<blocks_for(total, 256), 256, 0, s>>>(total, kRank * K, nodes, recv, mult);
    HIP_LAUNCH_CHECK();
}

// the one-collective exchange's pack / unpack (kernels.hpp OxArgs): one thread per
// double of the roots, then of the input positions, then of the multipole rows
template <bool PACK>
__device__ __forceinline__ void ox_element(const OxArgs& a, const int64_t e) {
    const int64_t nr = a.nRoot * a.rec, np = a.nPts * a.nb, nn = a.nNode * a.len;
    if (e < nr) {
        const int64_t j = e / a.rec, c = e - j * a.rec;
        if (PACK) a.buf[a.rootOff[j] + c] = a.roots[c];
        else a.roots[a.rootDst[j] + c] = a.buf[a.rootOff[j] + c];
    } else if (e < nr + np) {
        const int64_t t = e - nr, b = t / a.nPts, i = t - b * a.nPts;  // consecutive lanes: consecutive positions
        const int64_t q = a.base[i] + b * a.stride[i];
        if (PACK) a.buf[q] = a.x[(size_t)b * a.ldx + a.pos[i]];
        else a.x[(size_t)b * a.ldx + a.pos[i]] = a.buf[q];
    } else if (e < nr + np + nn) {
        const int64_t t = e - nr - np, j = t / a.len, c = t - j * a.len;
        if (PACK) a.buf[a.nodeBase[j] + c] = a.mult[(size_t)a.node[j] * a.len + c];
        else a.mult[(size_t)a.node[j] * a.len + c] = a.buf[a.nodeBase[j] + c];
    } else if (!PACK && a.ownRoots && e < nr + np + nn + a.rec) {
        const int64_t c = e - nr - np - nn;
        a.roots[a.ownDst + c] = a.ownRoots[c];
    } else if (!PACK && a.nSum > 0) {  // an upper node: its records summed in (rank, record) order
        const int64_t t = e - nr - np - nn - (a.ownRoots ? a.rec : 0), j = t / a.len, c = t - j * a.len;
        if (j >= a.nSum) return;
        // 8 records per round: their offsets, then their values, all loads of a round
        // independent (one dependent pair per record measured 16 us at 16 records)
        const int k0 = a.sumPtr[j], k1 = a.sumPtr[j + 1];
        double v = 0.0;
        for (int kb = k0; kb < k1; kb += 8) {
            int64_t o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = kb + u < k1 ? a.sumSrc[kb + u] : INT64_MIN;
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                x[u] = o[u] == INT64_MIN ? 0.0 : o[u] >= 0 ? a.buf[o[u] + c] : a.ownRec[~o[u] + c];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (kb + u < k1) v += x[u];
        }
        a.mult[(size_t)a.sumNode[j] * a.len + c] = v;
    }
}

template <bool PACK>
__global__ void k_ox(OxArgs a) {
    ox_element<PACK>(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Development (the loopback communicator, ANISO_LOOPBACK_XCHG_US): a stand-in for an
// exchange's latency on the stream -- `blocks` one-wave workgroups that each sleep
// until `us` microseconds of the 100 MHz real-time clock have passed (bounded: every
// wave exits), occupying a few CUs as the collective's kernels would.
__global__ void __launch_bounds__(64) k_spin_us(long long ticks) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void launch_spin_us(int us, int blocks, hipStream_t s) {
    if (us <= 0 || blocks <= 0) return;
    k_spin_us<<<blocks, 64, 0, s>>>((long long)us * 100);
    HIP_LAUNCH_CHECK();
}

void launch_ox(const OxArgs& a, bool pack, hipStream_t s) {
    const int64_t n = a.nRoot * a.rec + a.nPts * a.nb + a.nNode * a.len + (!pack && a.ownRoots ? a.rec : 0) +
                      (!pack ? a.nSum * a.len : 0);
    if (n <= 0) return;
    if (pack) k_ox<true><<<blocks_for(n, 256), 256, 0, s>>>(a);
    else k_ox<false><<<blocks_for(n, 256), 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
}

// The upper multipoles as partial sums (Plan::xUpTask), in the
// exchange's pack launch: its first workgroups take one partial task each -- this
// rank's tier-0 roots under one node A two levels above them.  M2M (bbfmm.h:855-859)
// of the roots to the mid level and to A, then A's contribution to each ancestor up
// to the topmost level an M2L reads, one transfer matrix per level.  M2M is linear,
// so this rank's share of an upper multipole is the M2M of its own roots alone; each
// share an M2L reads is a record, stored into this rank's record buffer and into
// every peer's part; the unpack sums every rank's records of a node in a fixed order
// (ox_element).  The other workgroups pack the input positions and multipole rows.
struct UpPack {
    int ntask = 0;
    const int* task = nullptr;  // Plan::kUpTaskInts ints per task
    const double* mult = nullptr;
    const Params* P = nullptr;
    double* rec = nullptr;            // this rank's records
    int nPeer = 0;
    const int64_t* peerOff = nullptr;  // each peer part's first record (doubles into the send buffer)
    int prio = 0;                      // raised wave priority for the task workgroups (ANISO_PACK_PRIO)
};

template <int K>
__global__ void __launch_bounds__(256) k_ox_pack_up(UpPack u, OxArgs a) {
    if ((int)blockIdx.x >= u.ntask) {
        ox_element<true>(a, (int64_t)(blockIdx.x - u.ntask) * blockDim.x + threadIdx.x);
        return;
    }
    __shared__ double sm[up_partial_lds<K>()];
    // the exchange waits on these few latency-bound workgroups, and the near field's own
    // groups run beside them: their waves issue first on a contended SIMD
    if (u.prio) __builtin_amdgcn_s_setprio(3);
    up_partial_task<K>(u.task + (size_t)blockIdx.x * Plan::kUpTaskInts, u.P, u.mult, u.rec, u.nPeer, u.peerOff, a.buf,
                       sm);
}

void launch_ox_pack_up(int K, int ntask, const int* task, const double* mult, const Params* P, double* rec,
                       int nPeer, const int64_t* peerOff, const OxArgs& a, hipStream_t s) {
    if (a.nRoot != 0) throw std::invalid_argument("pack with partial sums: the records replace the root parts");
    const int64_t n = a.nPts * a.nb + a.nNode * a.len;
    const unsigned nb = (unsigned)ntask + (unsigned)blocks_for(n, 256);
    if (nb == 0) return;
    // raised priority: 0.216 / 0.230 against 0.220 / 0.236 ms per rank of 8 (ranks 0 / 3,
    // r05zd); ANISO_PACK_PRIO=0 leaves it at the default
    static const int prio = [] {
        const char* e = std::getenv("ANISO_PACK_PRIO");
        return e ? std::atoi(e) : 1;
    }();
    const UpPack u{ntask, task, mult, P, rec, nPeer, peerOff, prio};
    ANISO_DISPATCH_K(K, (k_ox_pack_up<KK><<<nb, 256, 0, s>>>(u, a)));
    HIP_LAUNCH_CHECK();
}

void launch_m2l(int K, int ntgt, const int* tgt, const int64_t* ptr, const int* nDir, const int* canonBase,
                const int* outSlot, const int* src, const ModeArgs* tab, int nterm, const double* mult, int maxCanon,
                double* partial, double* local, hipStream_t s) {
    if (ntgt <= 0) return;
    if (maxCanon > kMaxCanon) throw std::invalid_argument("k_m2l: more canonical pairs per target than staged");
    const unsigned nb = blocks_for((int64_t)ntgt * kWave, 256);
    const size_t shm = K >= 4 ? (size_t)4 * std::max(maxCanon, 1) * kRank * K * sizeof(double) : 0;
    // blocks in flight per wave: 4 (8 KB) for one or two right-hand sides, 2 above
    ANISO_DISPATCH_K(K, (k_m2l<KK, (KK <= 2 ? 4 : 2)><<<nb, 256, shm, s>>>(ntgt, tgt, ptr, nDir, canonBase, outSlot,
                                                                            src, tab, nterm, mult, maxCanon, partial,
                                                                            local)));
    HIP_LAUNCH_CHECK();
}

void launch_m2l_gather(int K, int ntgt, const int* tgt, const int* inPtr, const double* partial, double* local,
                       hipStream_t s) {
    if (ntgt <= 0) return;
    const unsigned nb = blocks_for((int64_t)ntgt * kRank * K, 256);
    ANISO_DISPATCH_K(K, (k_m2l_gather<KK><<<nb, 256, 0, s>>>(ntgt, tgt, inPtr, partial, local)));
    HIP_LAUNCH_CHECK();
}

void launch_near_sym(int K, int nl, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts,
                     const int64_t* nearKOff, const int2* nearSym, const double* Kop, const double* fT,
                     const double* mix, const int* operm, int64_t obase, int64_t ldo, int maxS, int flags, double sgn,
                     double scale, int accum, double* partial, double* out, hipStream_t s) {
    if (nl <= 0) return;
    const int S = maxS > 0 ? maxS : 1;
    const int wpb = (size_t)S * K * 8 * 4 <= 48 * 1024 ? 4 : 1;  // waves per block, LDS = waves x S x K doubles
    const size_t shm = (size_t)wpb * S * K * sizeof(double);
    if (shm > 160 * 1024) throw std::invalid_argument("near field: leaf neighbourhood too large for LDS");
    ANISO_DISPATCH_K(K, (k_near_sym<KK><<<blocks_for(nl, wpb), wpb * kWave, shm, s>>>(
                            nl, leafInfo, nearPtsPtr, nearPts, nearKOff, nearSym, Kop, fT, make_mix<KK>(mix), operm,
                            obase, ldo, S, flags, sgn, scale, accum, partial, out)));
    HIP_LAUNCH_CHECK();
}

void launch_near(int K, int nl, int maxLeaf, const int4* leafInfo, const int64_t* nearPtsPtr, const int* nearPts,
                 const int64_t* nearKOff, const ModeArgs* tab, int nterm, const double* fT, const int* operm,
                 int64_t obase, int64_t ldo, int flags, double scale, int accum, double* out, hipStream_t s) {
    if (nl <= 0) return;
    if (maxLeaf <= 16) {  // 4 leaves per wave
        ANISO_DISPATCH_K(K, (k_near<KK, 16, 4><<<blocks_for((int64_t)nl * 16, 256), 256, 0, s>>>(
                                nl, leafInfo, nearPtsPtr, nearPts, nearKOff, tab, nterm, fT, operm, obase, ldo, flags,
                                scale, accum, out)));
    } else {
        ANISO_DISPATCH_K(K, (k_near<KK, 64, 4><<<blocks_for((int64_t)nl * 64, 256), 256, 0, s>>>(
                                nl, leafInfo, nearPtsPtr, nearPts, nearKOff, tab, nterm, fT, operm, obase, ldo, flags,
                                scale, accum, out)));
    }
    HIP_LAUNCH_CHECK();
}

void launch_down_tier(int K, int ntask, int maxTask, int maxLeaves, const int4* desc, const int* grpFix,
                      const int4* dn, const double* local, const Params* P, const int* leafSlot, const int* leafBegin,
                      const int2* leafNear, const double4* leafGeom, const double* pxT, const double* pyT,
                      const int* operm, int64_t obase, int64_t ldo, const int* nearOff, int maxNear,
                      const double* nearPart, const int2* chain, int maxChain, int flags, double scale, double* out,
                      const double* xsub, int64_t ldx, hipStream_t s, const double* hpart, const int* chainFold) {
    if (ntask <= 0) return;
    const size_t shm = down_tier_lds(maxTask, maxLeaves, maxNear, maxChain, K);
    ANISO_DISPATCH_K(K, (k_down_tier<KK><<<ntask, kTierThreads, shm, s>>>(
                            maxTask, maxLeaves, desc, grpFix, dn, local, P, leafSlot, leafBegin, leafNear, leafGeom,
                            pxT, pyT, operm, obase, ldo, nearOff, maxNear, nearPart, chain, maxChain, flags, scale,
                            out, xsub, ldx, hpart, chainFold)));
    HIP_LAUNCH_CHECK();
}

template <int D>
static void corr_d(int K, unsigned nb, int64_t b, int64_t e, const int* perm, const int* iperm, const double* cT,
                   const double* fT, const double* Wc, const double* Wm, const Params* P, int flags, double scale,
                   bool treeOut, int64_t ldo, double* out, hipStream_t s) {
    ANISO_DISPATCH_K(K, (k_corr<D, KK><<<nb, 256, 0, s>>>(b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut,
                                                          ldo, out)));
}

void launch_corr(int K, int d, int64_t b, int64_t e, const int* perm, const int* iperm, const double* cT,
                 const double* fT, const double* Wc, const double* Wm, const Params* P, int flags, double scale,
                 bool treeOut, int64_t ldo, double* out, hipStream_t s) {
    if (e <= b) return;
    const unsigned nb = blocks_for(e - b, 256);
    switch (d) {
        case 1: corr_d<1>(K, nb, b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut, ldo, out, s); break;
        case 2: corr_d<2>(K, nb, b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut, ldo, out, s); break;
        case 3: corr_d<3>(K, nb, b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut, ldo, out, s); break;
        case 4: corr_d<4>(K, nb, b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut, ldo, out, s); break;
        case 5: corr_d<5>(K, nb, b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut, ldo, out, s); break;
        case 6: corr_d<6>(K, nb, b, e, perm, iperm, cT, fT, Wc, Wm, P, flags, scale, treeOut, ldo, out, s); break;
        default: throw std::invalid_argument("quadRule out of range");
    }
    HIP_LAUNCH_CHECK();
}

}  // namespace aniso
