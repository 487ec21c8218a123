// f64op.hip -- the fp64 16-right-hand-side operator on MFMA (v_mfma_f64_16x16x4_f64):
// one mode's apply Y = K_id X (AnisoWrapper.cpp:92-136) or main.cpp's forward operator
// Y = X - K_0(sigma_s .* X) (main.cpp:125-136) for 16 right-hand sides at once, every
// FMM translation a dense 16 x 16 x 16 product on the fp64 matrix cores
// (DESIGN.md §3.16).  The same products as config 5's fp32 operator (f32op.hip):
//   P2M   mult[n]   = S_n (16 x pts) . F_pts (pts x 16)        bbfmm.h:737-748, 844
//   M2M   mult[p]  += R_q^T . mult[child q]                    bbfmm.h:855-859
//   M2L   local[t] += K_pair (16 x 16) . mult[src]             bbfmm.h:1051-1065
//   L2L   local[c] += R_q . local[parent]                      bbfmm.h:1070-1071
//   L2P   out_pts  += L_n (pts x 16) . local[n]                bbfmm.h:1104
//   near  out_pts  += K_near (pts x S) . F_src (S x 16)        bbfmm.h:1081-1099
// in fp64 with fp64 accumulation: the fp64 refinement of config 5 and 16-column
// batched mapping run here instead of two 8-right-hand-side VALU batches.
//
// Layouts (the fp64 MFMA's own accumulator order, MI355X: C/D element e of lane l is
// row (l >> 4) + 4e, column l & 15).  A node's 16 x 16 expansion (Chebyshev index x
// right-hand side) is kept in that order, 64 lanes x 32 B = 2 KB per node, one
// coalesced load or store.  Fed back as the B operand, element e of a lane is k-step
// e, whose k index for lane quarter h is h + 4e on both operands; an A operand is
// therefore stored "A order": element e of lane l = A[l & 15][(l >> 4) + 4e].  For a
// column-major 16 x 16 block (k_cache_m2l: s * 16 + t) that element sits at 64 e + l,
// so the fp64 M2L cache is rearranged in place, block by block, into lane-major
// 32-B rows (k64_lane_major).  Vectors are point-major N x 16 doubles in tree order.
#include <hip/hip_runtime.h>

#include <cmath>
#include <stdexcept>
#include <string>

#include "device_common.hpp"
#include "mrhs_corr.hpp"

namespace aniso {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// acc += A . B over k = 16: 4 MFMAs, step e taking element e of both fragments
__device__ __forceinline__ f64x4 mfma16_f64(const f64x4 a, const f64x4 b, f64x4 acc) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a.w, b.w, acc, 0, 0, 0);
    return acc;
}

__device__ __forceinline__ int wave_id64() {
    return __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave));
}

// P2M of every non-empty leaf (bbfmm.h:737-748, 844): mult[n] = S_n . F with the
// charges F = x (sigma_s) w formed here (AnisoWrapper.cpp:105-110); also stores
// them (fT: near field and stencil) and x (sigma_s) (cT: the singular term).
// sigT == nullptr: plain mapping (no sigma_s).
__global__ void __launch_bounds__(256) k64_p2m(int nleaf, const int* __restrict__ leaves,
                                               const int64_t* __restrict__ begin, const int64_t* __restrict__ count,
                                               const double* __restrict__ ncx, const double* __restrict__ ncy,
                                               const double* __restrict__ nrx, const double* __restrict__ nry,
                                               const double* __restrict__ pxT, const double* __restrict__ pyT,
                                               const double* __restrict__ X, const double* __restrict__ sigT,
                                               const double* __restrict__ wT, const Params* __restrict__ P,
                                               f64x4* __restrict__ mult, double* __restrict__ fT,
                                               double* __restrict__ cT) {
    const int w = wave_id64();
    if (w >= nleaf) return;
    const int lane = threadIdx.x & (kWave - 1), r = lane & 15, h = lane >> 4;
    const int n = leaves[w];
    const int64_t b = begin[n];
    const int cnt = (int)count[n];
    const double cx = ncx[n], cy = ncy[n], irx = 1.0 / nrx[n], iry = 1.0 / nry[n];
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int c0 = 0; c0 < cnt; c0 += 16) {
        f64x4 a, f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int p = c0 + h + 4 * e;  // k index of (step e, quarter h)
            const bool on = p < cnt;
            const int64_t pos = b + (on ? p : 0);
            double Sx[kNP], Sy[kNP];
            cheb_weights(P, (pxT[pos] - cx) * irx, Sx);
            cheb_weights(P, (pyT[pos] - cy) * iry, Sy);
            const double xv = X[pos * 16 + r];
            const double c = on ? (sigT ? xv * sigT[pos] : xv) : 0.0;
            const double fv = c * wT[pos];
            if (on) {
                fT[pos * 16 + r] = fv;
                cT[pos * 16 + r] = c;
            }
            a[e] = on ? Sx[r & 3] * Sy[r >> 2] : 0.0;  // A[cheb r][point]
            f[e] = fv;                                 // B[point][rhs r]
        }
        acc = mfma16_f64(a, f, acc);
    }
    mult[(size_t)n * 64 + lane] = acc;
}

// M2M of one level (bbfmm.h:855-859): mult[p] = sum over non-empty children q of R_q^T mult[q]
__global__ void __launch_bounds__(256) k64_m2m(int nn, const int* __restrict__ nodes, const int4* __restrict__ child,
                                               const int64_t* __restrict__ count, const f64x4* __restrict__ Rup,
                                               f64x4* __restrict__ mult) {
    const int w = wave_id64();
    if (w >= nn) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int n = nodes[w];
    const int4 c = child[n];
    const int ch[4] = {c.x, c.y, c.z, c.w};
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (count[ch[q]] == 0) continue;  // wave-uniform
        acc = mfma16_f64(Rup[q * 64 + lane], mult[(size_t)ch[q] * 64 + lane], acc);
    }
    mult[(size_t)n * 64 + lane] = acc;
}

// M2L over V then X (bbfmm.h:1051-1065): local[t] = sum over its directed pairs of
// K_pair . mult[src]; the pair's block is 2 KB in A order (one f64x4 per lane).
// Two accumulators (one pair's MFMA chain is 4 deep) and two pairs in flight.
__global__ void __launch_bounds__(256) k64_m2l(int ntgt, const int* __restrict__ tgt, const int64_t* __restrict__ ptr,
                                               const int* __restrict__ src, const f64x4* __restrict__ K64,
                                               const f64x4* __restrict__ mult, f64x4* __restrict__ local) {
    const int w = wave_id64();
    if (w >= ntgt) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t p0 = ptr[w], p1 = ptr[w + 1];
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    int64_t p = p0;
    for (; p + 1 < p1; p += 2) {
        const int s0 = src[p], s1 = src[p + 1];
        const f64x4 a0 = __builtin_nontemporal_load(K64 + (size_t)p * 64 + lane);
        const f64x4 a1 = __builtin_nontemporal_load(K64 + (size_t)(p + 1) * 64 + lane);
        const f64x4 b0 = mult[(size_t)s0 * 64 + lane], b1 = mult[(size_t)s1 * 64 + lane];
        acc0 = mfma16_f64(a0, b0, acc0);
        acc1 = mfma16_f64(a1, b1, acc1);
    }
    if (p < p1)
        acc0 = mfma16_f64(__builtin_nontemporal_load(K64 + (size_t)p * 64 + lane), mult[(size_t)src[p] * 64 + lane],
                          acc0);
    local[(size_t)tgt[w] * 64 + lane] = acc0 + acc1;
}

// L2L of one level (bbfmm.h:1070-1071): local[n] += R_slot(n) . local[parent]
__global__ void __launch_bounds__(256) k64_l2l(int nn, const int* __restrict__ nodes, const int* __restrict__ parent,
                                               const int* __restrict__ slot, const f64x4* __restrict__ Rdn,
                                               f64x4* __restrict__ local) {
    const int w = wave_id64();
    if (w >= nn) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int n = nodes[w];
    f64x4 acc = local[(size_t)n * 64 + lane];
    acc = mfma16_f64(Rdn[slot[n] * 64 + lane], local[(size_t)parent[n] * 64 + lane], acc);
    local[(size_t)n * 64 + lane] = acc;
}

// Per leaf: L2P (bbfmm.h:1104) and the U/W near field (bbfmm.h:1081-1099) as MFMA
// tiles of 16 target points; Y = scale (far + near) (mapping) or X - scale (far +
// near) (forward).  Near tiles: per (row block, 16 source columns) 64 lanes x f64x4,
// element e of lane l = K[row 16 rb + (l&15)][col 16 s4 + (l>>4) + 4e]; the source
// list is padded to a multiple of 16 (zero columns).
__global__ void __launch_bounds__(256) k64_leaf(int nleaf, const int4* __restrict__ leafInfo,
                                                const int64_t* __restrict__ nearPtr, const int* __restrict__ nearPts,
                                                const int64_t* __restrict__ koff, const f64x4* __restrict__ Knear,
                                                const int* __restrict__ level, const double* __restrict__ ncx,
                                                const double* __restrict__ ncy, const double* __restrict__ nrx,
                                                const double* __restrict__ nry, const double* __restrict__ pxT,
                                                const double* __restrict__ pyT, const Params* __restrict__ P,
                                                const f64x4* __restrict__ local, const double* __restrict__ fT,
                                                const double* __restrict__ X, double scale, int flags,
                                                double* __restrict__ Y) {
    const int w = wave_id64();
    if (w >= nleaf) return;
    const int lane = threadIdx.x & (kWave - 1), r = lane & 15, h = lane >> 4;
    const int4 info = leafInfo[w];  // node, begin, count, padded sources
    const int n = info.x, cnt = info.z, Sp = (flags & kStageNear) ? info.w : 0;
    const int64_t b = info.y, pb = nearPtr[w];
    const bool far = (flags & kStageFar) && level[n] >= 1;  // the root's local is zero
    const f64x4 loc = far ? local[(size_t)n * 64 + lane] : f64x4{0.0, 0.0, 0.0, 0.0};
    const double cx = ncx[n], cy = ncy[n], irx = 1.0 / nrx[n], iry = 1.0 / nry[n];
    const int nst4 = Sp >> 4, nrb = (cnt + 15) >> 4;
    for (int rb = 0; rb < nrb; ++rb) {
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        if (far) {  // A[point 16 rb + r][cheb h + 4e] = L_cheb(point)
            const int p = 16 * rb + r;
            const int64_t pos = b + min(p, cnt - 1);
            double Sx[kNP], Sy[kNP];
            cheb_weights(P, (pxT[pos] - cx) * irx, Sx);
            cheb_weights(P, (pyT[pos] - cy) * iry, Sy);
            f64x4 a;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = h + 4 * e;
                a[e] = p < cnt ? Sx[k & 3] * Sy[k >> 2] : 0.0;
            }
            acc = mfma16_f64(a, loc, acc);
        }
        const f64x4* kt = Knear + koff[w] + (size_t)rb * nst4 * 64 + lane;
        for (int s4 = 0; s4 < nst4; ++s4) {
            const f64x4 a = __builtin_nontemporal_load(kt + (size_t)s4 * 64);
            f64x4 f;
#pragma unroll
            for (int e = 0; e < 4; ++e) f[e] = fT[(size_t)nearPts[pb + 16 * s4 + h + 4 * e] * 16 + r];
            acc = mfma16_f64(a, f, acc);
        }
        const bool fwd = (flags & kStageForward) != 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // lane: points 16 rb + h + 4e, right-hand side r
            const int p = 16 * rb + h + 4 * e;
            if (p < cnt) {
                const int64_t pos = b + p;
                Y[pos * 16 + r] = fwd ? X[pos * 16 + r] - scale * acc[e] : scale * acc[e];
            }
        }
    }
}

// The fp64 column-major M2L blocks (k_cache_m2l: pair * 256 + s * 16 + t) rearranged
// in place into A order, lane-major (element e of lane l = K[t = l&15][s = (l>>4) +
// 4e] = block[64 e + l] moves to block[4 l + e]): one wave per block.
__global__ void __launch_bounds__(256) k64_lane_major(int64_t npairs, double* __restrict__ K) {
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (w >= npairs) return;
    const int lane = threadIdx.x & (kWave - 1);
    double* blk = K + (size_t)w * 256;
    f64x4 v;  // the store needs all four loads of every lane: no lane overwrites unread data
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = blk[64 * e + lane];
    reinterpret_cast<f64x4*>(blk)[lane] = v;
}

// near blocks of one leaf (k_cache_near: nT4 x S column-major, rows padded to 4) ->
// fp64 tiles (k64_leaf)
__global__ void k64_conv_near(int nl, const int4* __restrict__ info, const int64_t* __restrict__ koffD,
                              const int64_t* __restrict__ koff, const int* __restrict__ srcCount,
                              const double* __restrict__ Kd, double* __restrict__ K64) {
    const int li = blockIdx.y;
    if (li >= nl) return;
    const int4 in = info[li];
    const int nT = in.z, Sp = in.w, S = srcCount[li];
    const int nT4 = (nT + 3) & ~3, nrb = (nT + 15) >> 4, nst4 = Sp >> 4;
    const int64_t total = (int64_t)nrb * nst4 * 256;
    double* dst = K64 + koff[li] * 4;
    const double* src = Kd + koffD[li];
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(id & 3), l = (int)((id >> 2) & 63);
        const int64_t tile = id >> 8;
        const int s4 = (int)(tile % nst4), rb = (int)(tile / nst4);
        const int t = 16 * rb + (l & 15), s = 16 * s4 + (l >> 4) + 4 * e;
        dst[id] = (t < nT && s < S) ? src[(int64_t)s * nT4 + t] : 0.0;
    }
}

// ----------------------------------------------------------------- launchers

void launch64_p2m(int nleaf, const int* leaves, const int64_t* begin, const int64_t* count, const double* ncx,
                  const double* ncy, const double* nrx, const double* nry, const double* pxT, const double* pyT,
                  const double* X, const double* sigT, const double* wT, const Params* P, void* mult, double* fT,
                  double* cT, hipStream_t s) {
    if (nleaf <= 0) return;
    k64_p2m<<<blocks_for((int64_t)nleaf * kWave, 256), 256, 0, s>>>(nleaf, leaves, begin, count, ncx, ncy, nrx, nry,
                                                                   pxT, pyT, X, sigT, wT, P,
                                                                   static_cast<f64x4*>(mult), fT, cT);
    HIP_LAUNCH_CHECK();
}

void launch64_m2m(int nn, const int* nodes, const int4* child, const int64_t* count, const void* Rup, void* mult,
                  hipStream_t s) {
    if (nn <= 0) return;
    k64_m2m<<<blocks_for((int64_t)nn * kWave, 256), 256, 0, s>>>(nn, nodes, child, count,
                                                                static_cast<const f64x4*>(Rup),
                                                                static_cast<f64x4*>(mult));
    HIP_LAUNCH_CHECK();
}

void launch64_m2l(int ntgt, const int* tgt, const int64_t* ptr, const int* src, const void* K64, const void* mult,
                  void* local, hipStream_t s) {
    if (ntgt <= 0) return;
    k64_m2l<<<blocks_for((int64_t)ntgt * kWave, 256), 256, 0, s>>>(ntgt, tgt, ptr, src, static_cast<const f64x4*>(K64),
                                                                  static_cast<const f64x4*>(mult),
                                                                  static_cast<f64x4*>(local));
    HIP_LAUNCH_CHECK();
}

void launch64_l2l(int nn, const int* nodes, const int* parent, const int* slot, const void* Rdn, void* local,
                  hipStream_t s) {
    if (nn <= 0) return;
    k64_l2l<<<blocks_for((int64_t)nn * kWave, 256), 256, 0, s>>>(nn, nodes, parent, slot,
                                                                static_cast<const f64x4*>(Rdn),
                                                                static_cast<f64x4*>(local));
    HIP_LAUNCH_CHECK();
}

void launch64_leaf(int nleaf, const int4* leafInfo, const int64_t* nearPtr, const int* nearPts, const int64_t* koff,
                   const void* Knear, const int* level, const double* ncx, const double* ncy, const double* nrx,
                   const double* nry, const double* pxT, const double* pyT, const Params* P, const void* local,
                   const double* fT, const double* X, double scale, int flags, double* Y, hipStream_t s) {
    if (nleaf <= 0) return;
    k64_leaf<<<blocks_for((int64_t)nleaf * kWave, 256), 256, 0, s>>>(
        nleaf, leafInfo, nearPtr, nearPts, koff, static_cast<const f64x4*>(Knear), level, ncx, ncy, nrx, nry, pxT,
        pyT, P, static_cast<const f64x4*>(local), fT, X, scale, flags, Y);
    HIP_LAUNCH_CHECK();
}

void launch64_corr(int d, int64_t N, const int* perm, const int* iperm, const double* cT, const double* fT,
                   const double* C, const double* mu, const Params* P, int flags, double scale, double* Y,
                   hipStream_t s) {
    if (N <= 0) return;
    const unsigned nb = blocks_for(N, 256);
    switch (d) {
        case 1: k16_corr<double, 1><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 2: k16_corr<double, 2><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 3: k16_corr<double, 3><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 4: k16_corr<double, 4><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 5: k16_corr<double, 5><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 6: k16_corr<double, 6><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        default: throw std::invalid_argument("quadRule out of range");
    }
    HIP_LAUNCH_CHECK();
}

void launch64_lane_major(int64_t npairs, double* K, hipStream_t s) {
    if (npairs <= 0) return;
    k64_lane_major<<<blocks_for(npairs * kWave, 256), 256, 0, s>>>(npairs, K);
    HIP_LAUNCH_CHECK();
}

// k <= 16 columns of an original-order N x k column-major block -> point-major tree
// order N x 16 (zero columns beyond k), and back (aniso_mapping_batched)
__global__ void k64_gather16(int64_t N, int k, const int* __restrict__ perm, const double* __restrict__ Q,
                             double* __restrict__ X16) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= N * 16) return;
    const int64_t pos = id >> 4;
    const int j = (int)(id & 15);
    X16[id] = j < k ? Q[(size_t)j * N + perm[pos]] : 0.0;
}

__global__ void k64_scatter16(int64_t N, int k, const int* __restrict__ perm, const double* __restrict__ Y16,
                              double* __restrict__ Out) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= N * 16) return;
    const int64_t pos = id >> 4;
    const int j = (int)(id & 15);
    if (j < k) Out[(size_t)j * N + perm[pos]] = Y16[id];
}

void launch64_gather16(int64_t N, int k, const int* perm, const double* Q, double* X16, hipStream_t s) {
    k64_gather16<<<blocks_for(N * 16, 256), 256, 0, s>>>(N, k, perm, Q, X16);
    HIP_LAUNCH_CHECK();
}

void launch64_scatter16(int64_t N, int k, const int* perm, const double* Y16, double* Out, hipStream_t s) {
    k64_scatter16<<<blocks_for(N * 16, 256), 256, 0, s>>>(N, k, perm, Y16, Out);
    HIP_LAUNCH_CHECK();
}

void launch64_conv_near(int nl, const int4* info, const int64_t* koffD, const int64_t* koff, const int* srcCount,
                        const double* Kd, void* K64, hipStream_t s) {
    if (nl <= 0) return;
    dim3 grid(4, (unsigned)nl);
    k64_conv_near<<<grid, 256, 0, s>>>(nl, info, koffD, koff, srcCount, Kd, static_cast<double*>(K64));
    HIP_LAUNCH_CHECK();
}

}  // namespace aniso
