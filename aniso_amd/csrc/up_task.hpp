// up_task.hpp -- one up-pass task (P2M of its leaves, M2M of its levels), shared by
// the tier launches (apply.hip k_up_tier) and the fused top-of-tree + M2L launch
// (harmonic.hip k_top_m2l_hc).
#pragma once

#include "device_common.hpp"
#include "host.hpp"  // kTaskLevels, kLeafCode

namespace aniso {

// Base charge b of tree position k: x_tree[b][k] (treeIn) or x[b][perm[k]], times
// sigma_s in tree order when given.
__device__ __forceinline__ double input_charge(const double* __restrict__ xin, int64_t ldi, int b, int treeIn,
                                               const int* __restrict__ perm, const double* __restrict__ sigT,
                                               int64_t k) {
    const double c = xin[(size_t)b * ldi + (treeIn ? k : (int64_t)perm[k])];
    return sigT ? c * sigT[k] : c;
}

// Up pass (bbfmm.h:825-861) as tiers of <= 4-level subtrees:
// one workgroup per subtree keeps its nodes' multipoles in LDS, deepest level
// first; a leaf's multipole is P2M over its contiguous tree-order points
// (bbfmm.h:737-748), an internal node's is M2M of its children (bbfmm.h:855-859),
// where a child below the tier is the root of a lower tier's task (read from HBM).
// Phase 0 stages the transfer matrices, node boxes and child codes in LDS with
// one round of independent loads; the levels then run out of LDS.
// 16-lane reduce-scatter of acc[2 NV] (P2M): lane ln keeps half, adds the partner's half
#define ANISO_RS16(NV, OFF)                                        \
    {                                                              \
        const bool hi = ln & (OFF);                                \
        _Pragma("unroll") for (int e = 0; e < (NV); ++e) {         \
            const double keep = hi ? acc[e + (NV)] : acc[e];       \
            const double send = hi ? acc[e] : acc[e + (NV)];       \
            acc[e] = keep + xor16_f64<(OFF)>(send, r4);            \
        }                                                          \
    }
// One up task (workgroup-wide).  rootSlot / recv (sharded applies, may be null):
// a child that is a tier-0 root with rootSlot >= 0 is read from the all-gathered
// records recv[rootSlot] (and copied to mult for the M2L) instead of mult.
template <int K>
__device__ __forceinline__ void up_task(
    int task, int maxTask, const int4* __restrict__ desc, const int* __restrict__ grpFix,
    const int* __restrict__ node, const int4* __restrict__ code, const double4* __restrict__ geom,
    const int2* __restrict__ leafRange, const double* __restrict__ pxT, const double* __restrict__ pyT,
    const double* __restrict__ xin, int64_t ldi, int treeIn, const int* __restrict__ perm,
    const double* __restrict__ sigT, const double* __restrict__ wT, double* __restrict__ fT, double* __restrict__ cT,
    const Params* __restrict__ P, double* __restrict__ mult, const int* __restrict__ rootSlot,
    const double* __restrict__ recv, const int* __restrict__ sendSlot, double* __restrict__ send, double* sm) {
    int4* CD = reinterpret_cast<int4*>(sm);                // maxTask child codes
    double* Rl = reinterpret_cast<double*>(CD + maxTask);  // 4 x 256 transfer matrices (transposed)
    double* M = Rl + 4 * kRank * kRank;                    // maxTask x 16 x K multipoles
    double* G = M + (size_t)maxTask * kRank * K;           // maxTask x 4: cx, cy, 1/rx, 1/ry
    int* LB = reinterpret_cast<int*>(G + (size_t)maxTask * 4);  // maxTask: leaf point offset, count, node
    int* LC = LB + maxTask;
    int* ND = LC + maxTask;
    int* RS = ND + maxTask;  // recv: per (node, child) the gathered record slot of a tier-0 root child (-1: none)
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
    if (recv) {
        // the gathered tier-0 roots under this task: their record slots in one round of
        // independent loads, then the records stored for the M2L (all lanes, coalesced;
        // the slot lookup inside the copy loop made every iteration two dependent
        // round trips: 42 us per 5-node task on a rank of 8, r04ab)
        for (int i = threadIdx.x; i < nt * 4; i += blockDim.x) {
            const int4 c = CD[i >> 2];
            const int q = i & 3;
            const int cq = q == 0 ? c.x : q == 1 ? c.y : q == 2 ? c.z : c.w;
            RS[i] = (c.x == kLeafCode || cq >= -1) ? -1 : rootSlot[-cq - 2];
        }
        __syncthreads();
        constexpr int RK = kRank * K;
        for (int it = threadIdx.x; it < nt * 4 * RK; it += blockDim.x) {
            const int i = it / RK, e = it - i * RK;
            const int rs = RS[i];
            if (rs < 0) continue;
            const int4 c = CD[i >> 2];
            const int q = i & 3;
            const int cq = q == 0 ? c.x : q == 1 ? c.y : q == 2 ? c.z : c.w;
            mult[(size_t)(-cq - 2) * RK + e] = recv[(size_t)rs * RK + e];
        }
    }
    // P2M of the task's leaves (bbfmm.h:737-748): 16 lanes per leaf, one point per
    // lane per pass (its 16 products in registers), then a 16-lane reduce-scatter
    // leaves lane l with entry l.  The weighted charges are formed here from the
    // apply's input (the reference's charge .* weights, AnisoWrapper.cpp:105-110).
    {
        const int gi = threadIdx.x >> 4, ln = threadIdx.x & 15, ngr = blockDim.x >> 4;
        const bool r4 = xor16_r4((int)threadIdx.x);  // DPP rotate for the xor-4 step
        for (int k = gi; k < nt; k += ngr) {
            if (CD[k].x != kLeafCode) continue;  // uniform over the 16 lanes
            const double cx = G[4 * k], cy = G[4 * k + 1], irx = G[4 * k + 2], iry = G[4 * k + 3];
            const int pe = LB[k] + LC[k];
            if (LC[k] <= 16) {  // one point per lane: its Chebyshev weights once for all K base vectors
                const int p = LB[k] + ln;
                const bool on = p < pe;
                const int64_t kp = b0 + (on ? p : LB[k]);
                double Sx[kNP], Sy[kNP], cb[K];
                cheb_weights(P, (pxT[kp] - cx) * irx, Sx);
                cheb_weights(P, (pyT[kp] - cy) * iry, Sy);
                const double w = wT[kp];
                double fb[K];
#pragma unroll
                for (int b = 0; b < K; ++b) {
                    cb[b] = input_charge(xin, ldi, b, treeIn, perm, sigT, kp);
                    fb[b] = on ? cb[b] * w : 0.0;
                }
                if (on && fT) {  // for the near field and the corrections (fT null: they read the input)
                    store_charges<K>(fT + kp * kStride<K>, fb);
                    store_charges<K>(cT + kp * kStride<K>, cb);
                }
#pragma unroll
                for (int b = 0; b < K; ++b) {
                    const double f = fb[b];
                    double acc[kRank];
#pragma unroll
                    for (int j = 0; j < kNP; ++j) {
                        const double sf = Sy[j] * f;
#pragma unroll
                        for (int i = 0; i < kNP; ++i) acc[j * kNP + i] = Sx[i] * sf;
                    }
                    ANISO_RS16(8, 8)
                    ANISO_RS16(4, 4)
                    ANISO_RS16(2, 2)
                    ANISO_RS16(1, 1)
                    M[((size_t)k * kRank + ln) * K + b] = acc[0];
                }
                continue;
            }
#pragma unroll 1
            for (int b = 0; b < K; ++b) {
                double acc[kRank];
#pragma unroll
                for (int e = 0; e < kRank; ++e) acc[e] = 0.0;
                for (int p = LB[k] + ln; p < pe; p += 16) {
                    const int64_t kp = b0 + p;
                    const double c = input_charge(xin, ldi, b, treeIn, perm, sigT, kp);
                    const double f = c * wT[kp];
                    if (fT) {  // for k_near and the corrections
                        fT[kp * kStride<K> + b] = f;
                        cT[kp * kStride<K> + b] = c;
                    }
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
                ANISO_RS16(8, 8)
                ANISO_RS16(4, 4)
                ANISO_RS16(2, 2)
                ANISO_RS16(1, 1)
                M[((size_t)k * kRank + ln) * K + b] = acc[0];
            }
        }
    }
    __syncthreads();
    // M2M (bbfmm.h:855-859), one item per (node, row r, child q): 4x the items of a
    // per-(node, row) loop, so a level's child reads (LDS, or HBM for the roots of
    // the tier below) are all in flight at once; the 4 child partials of a row are
    // adjacent lanes, summed by a DPP quad reduction in a fixed order.
    for (int g = 0; g < ngrp; ++g) {
        const int s0 = gs[g], s1 = gs[g + 1];
        for (int it = threadIdx.x; it < (s1 - s0) * kRank * 4; it += blockDim.x) {
            const int k = s0 + (it >> 6), r = (it >> 2) & (kRank - 1), q = it & 3;
            const int4 c = CD[k];
            const int cq = q == 0 ? c.x : q == 1 ? c.y : q == 2 ? c.z : c.w;
            double acc[K];
#pragma unroll
            for (int b = 0; b < K; ++b) acc[b] = 0.0;
            if (c.x != kLeafCode && cq != -1) {
                const double* R = Rl + q * kRank * kRank + r;  // transposed: R[rr * 16 + r]
                const double* cm = M + (size_t)(cq >= 0 ? cq : 0) * kRank * K;  // child in this task (LDS)
                if (cq < 0) {  // root of the tier below: HBM (or the gathered records)
                    const int rs = recv ? RS[4 * k + q] : -1;
                    cm = rs >= 0 ? recv + (size_t)rs * kRank * K : mult + (size_t)(-cq - 2) * kRank * K;
                }
#pragma unroll
                for (int rr = 0; rr < kRank; ++rr)
#pragma unroll
                    for (int b = 0; b < K; ++b) acc[b] += R[rr * kRank] * cm[rr * K + b];
            }
#pragma unroll
            for (int b = 0; b < K; ++b) acc[b] = quad_sum(acc[b]);
            if (q == 0 && c.x != kLeafCode) {  // leaves: P2M above
#pragma unroll
                for (int b = 0; b < K; ++b) M[((size_t)k * kRank + r) * K + b] = acc[b];
            }
        }
        __syncthreads();
    }
    for (int it = threadIdx.x; it < nt * kRank * K; it += blockDim.x)
        mult[(size_t)ND[it / (kRank * K)] * kRank * K + it % (kRank * K)] = M[it];
    if (send) {  // sharded bottom tier: the task root's record into this rank's all-gather buffer
        const int ss = sendSlot[ND[nt - 1]];  // the root is the task's last node (deepest level first)
        if (ss >= 0)
            for (int e = threadIdx.x; e < kRank * K; e += blockDim.x)
                send[(size_t)ss * kRank * K + e] = M[(size_t)(nt - 1) * kRank * K + e];
    }
}

#undef ANISO_RS16

}  // namespace aniso
