// f32op.hip -- config 5's fp32 operator on MFMA: main.cpp's forward operator
// Y = X - K_0(sigma_s .* X) (main.cpp:125-136) for 16 right-hand sides at once, with
// the operator caches in fp32.
//
// With 16 right-hand sides every FMM translation of one node is a dense 16 x 16 x 16
// product -- the matrix shape of v_mfma_f32_16x16x4_f32 (4 instructions per
// product):
//   P2M   mult[n]   = S_n (16 x pts) . F_pts (pts x 16)        bbfmm.h:737-748, 844
//   M2M   mult[p]  += R_q^T . mult[child q]                    bbfmm.h:855-859
//   M2L   local[t] += K_pair (16 x 16) . mult[src]             bbfmm.h:1051-1065
//   L2L   local[c] += R_q . local[parent]                      bbfmm.h:1070-1071
//   L2P   out_pts  += L_n (pts x 16) . local[n]                bbfmm.h:1104
//   near  out_pts  += K_near (pts x S) . F_src (S x 16)        bbfmm.h:1081-1099
// One wave per node (or leaf), fp32 in, fp32 accumulate (exact fp32 MFMA).
//
// Layouts.  A node's 16 x 16 expansion (Chebyshev index x right-hand side) is kept
// in the MFMA accumulator order "F": lane l holds rows 4(l>>4) .. 4(l>>4)+3 of
// column l&15 (64 lanes x float4 = 1 KB per node, one coalesced load or store).
// Fed back as the B operand, element e of a lane is the k-step e of that lane's k
// quarter: the k index of (step e, lane quarter h) is 4h + e on both operands, so
// an A operand is stored as A[l&15][4(l>>4) .. +3] per lane (float4, lane-major).
// Point-major vectors: X[pos][16] in tree order (the 16 right-hand sides of one
// point are one 64-B line).
#include <hip/hip_runtime.h>

#include <cmath>
#include <stdexcept>
#include <string>

#include "device_common.hpp"
#include "mrhs_corr.hpp"

namespace aniso {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// acc += A . B over k = 16: 4 MFMAs, step e taking element e of both fragments
__device__ __forceinline__ f32x4 mfma16(const f32x4 a, const f32x4 b, f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
    return acc;
}

__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave));
}

// Chebyshev weights S(s, c_i), i < 4, of the scaled coordinate s (device_common.hpp)
__device__ __forceinline__ void cheb4(const Params* __restrict__ P, double s, double (&S)[kNP]) {
    cheb_weights(P, s, S);
}

// P2M of every non-empty leaf (bbfmm.h:737-748, 844): mult[n] = S_n . F with the
// charges F = x sigma_s w formed here (AnisoWrapper.cpp:105-110); also stores them
// (fT: the near field and the stencil read them) and x sigma_s (cT: the singular term).
__global__ void __launch_bounds__(256) k32_p2m(int nleaf, const int* __restrict__ leaves,
                                               const int64_t* __restrict__ begin, const int64_t* __restrict__ count,
                                               const double* __restrict__ ncx, const double* __restrict__ ncy,
                                               const double* __restrict__ nrx, const double* __restrict__ nry,
                                               const double* __restrict__ pxT, const double* __restrict__ pyT,
                                               const float* __restrict__ X, const double* __restrict__ sigT,
                                               const double* __restrict__ wT, const Params* __restrict__ P,
                                               f32x4* __restrict__ mult, float* __restrict__ fT,
                                               float* __restrict__ cT) {
    const int w = wave_id();
    if (w >= nleaf) return;
    const int lane = threadIdx.x & (kWave - 1), r = lane & 15, h = lane >> 4;
    const int n = leaves[w];
    const int64_t b = begin[n];
    const int cnt = (int)count[n];
    const double cx = ncx[n], cy = ncy[n], irx = 1.0 / nrx[n], iry = 1.0 / nry[n];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < cnt; c0 += 16) {
        f32x4 a, f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int p = c0 + 4 * h + e;
            const bool on = p < cnt;
            const int64_t pos = b + (on ? p : 0);
            double Sx[kNP], Sy[kNP];
            cheb4(P, (pxT[pos] - cx) * irx, Sx);
            cheb4(P, (pyT[pos] - cy) * iry, Sy);
            const double c = on ? (double)X[pos * 16 + r] * sigT[pos] : 0.0;
            const double fv = c * wT[pos];
            if (on) {
                fT[pos * 16 + r] = (float)fv;
                cT[pos * 16 + r] = (float)c;
            }
            a[e] = on ? (float)(Sx[r & 3] * Sy[r >> 2]) : 0.f;  // A[cheb r][point]
            f[e] = (float)fv;                                  // B[point][rhs r]
        }
        acc = mfma16(a, f, acc);
    }
    mult[(size_t)n * 64 + lane] = acc;
}

// M2M of one level (bbfmm.h:855-859): mult[p] = sum over non-empty children q of R_q^T mult[q]
__global__ void __launch_bounds__(256) k32_m2m(int nn, const int* __restrict__ nodes, const int4* __restrict__ child,
                                               const int64_t* __restrict__ count, const f32x4* __restrict__ Rup,
                                               f32x4* __restrict__ mult) {
    const int w = wave_id();
    if (w >= nn) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int n = nodes[w];
    const int4 c = child[n];
    const int ch[4] = {c.x, c.y, c.z, c.w};
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (count[ch[q]] == 0) continue;  // wave-uniform
        acc = mfma16(Rup[q * 64 + lane], mult[(size_t)ch[q] * 64 + lane], acc);
    }
    mult[(size_t)n * 64 + lane] = acc;
}

// M2L over V then X (bbfmm.h:1051-1065): local[t] = sum over its directed pairs of
// K_pair . mult[src]; the pair's fp32 block is 1 KB in A order (one float4 per lane).
// Two accumulators (the MFMA chain of one pair is 4 deep) and two pairs in flight.
__global__ void __launch_bounds__(256) k32_m2l(int ntgt, const int* __restrict__ tgt, const int64_t* __restrict__ ptr,
                                               const int* __restrict__ src, const f32x4* __restrict__ K32,
                                               const f32x4* __restrict__ mult, f32x4* __restrict__ local) {
    const int w = wave_id();
    if (w >= ntgt) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t p0 = ptr[w], p1 = ptr[w + 1];
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    int64_t p = p0;
    for (; p + 1 < p1; p += 2) {
        const int s0 = src[p], s1 = src[p + 1];
        const f32x4 a0 = __builtin_nontemporal_load(K32 + (size_t)p * 64 + lane);
        const f32x4 a1 = __builtin_nontemporal_load(K32 + (size_t)(p + 1) * 64 + lane);
        const f32x4 b0 = mult[(size_t)s0 * 64 + lane], b1 = mult[(size_t)s1 * 64 + lane];
        acc0 = mfma16(a0, b0, acc0);
        acc1 = mfma16(a1, b1, acc1);
    }
    if (p < p1) acc0 = mfma16(__builtin_nontemporal_load(K32 + (size_t)p * 64 + lane), mult[(size_t)src[p] * 64 + lane], acc0);
    local[(size_t)tgt[w] * 64 + lane] = acc0 + acc1;
}

// L2L of one level (bbfmm.h:1070-1071): local[n] += R_slot(n) . local[parent]
__global__ void __launch_bounds__(256) k32_l2l(int nn, const int* __restrict__ nodes, const int* __restrict__ parent,
                                               const int* __restrict__ slot, const f32x4* __restrict__ Rdn,
                                               f32x4* __restrict__ local) {
    const int w = wave_id();
    if (w >= nn) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int n = nodes[w];
    f32x4 acc = local[(size_t)n * 64 + lane];
    acc = mfma16(Rdn[slot[n] * 64 + lane], local[(size_t)parent[n] * 64 + lane], acc);
    local[(size_t)n * 64 + lane] = acc;
}

// Per leaf: L2P (bbfmm.h:1104) and the U/W near field (bbfmm.h:1081-1099) as
// MFMA tiles of 16 target points, then Y = X - scale (far + near).  The near
// blocks are fp32 tiles: per (row block, 16 source columns) 64 lanes x float4,
// element e of lane l = K[row 16 rb + (l&15)][col 16 s4 + 4e + (l>>4)]; the source
// list is padded to a multiple of 16 (zero columns).
__global__ void __launch_bounds__(256) k32_leaf(int nleaf, const int4* __restrict__ leafInfo,
                                                const int64_t* __restrict__ nearPtr, const int* __restrict__ nearPts,
                                                const int64_t* __restrict__ koff, const f32x4* __restrict__ Knear,
                                                const int* __restrict__ level, const double* __restrict__ ncx,
                                                const double* __restrict__ ncy, const double* __restrict__ nrx,
                                                const double* __restrict__ nry, const double* __restrict__ pxT,
                                                const double* __restrict__ pyT, const Params* __restrict__ P,
                                                const f32x4* __restrict__ local, const float* __restrict__ fT,
                                                const float* __restrict__ X, float scale, int flags,
                                                float* __restrict__ Y) {
    const int w = wave_id();
    if (w >= nleaf) return;
    const int lane = threadIdx.x & (kWave - 1), r = lane & 15, h = lane >> 4;
    const int4 info = leafInfo[w];  // node, begin, count, padded sources
    const int n = info.x, cnt = info.z, Sp = (flags & kStageNear) ? info.w : 0;
    const int64_t b = info.y, pb = nearPtr[w];
    const bool far = (flags & kStageFar) && level[n] >= 1;  // the root's local is zero
    const f32x4 loc = far ? local[(size_t)n * 64 + lane] : f32x4{0.f, 0.f, 0.f, 0.f};
    const double cx = ncx[n], cy = ncy[n], irx = 1.0 / nrx[n], iry = 1.0 / nry[n];
    const int nst4 = Sp >> 4, nrb = (cnt + 15) >> 4;
    for (int rb = 0; rb < nrb; ++rb) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (far) {  // A[point 16 rb + r][cheb 4h + e] = L_cheb(point)
            const int p = 16 * rb + r;
            const int64_t pos = b + min(p, cnt - 1);
            double Sx[kNP], Sy[kNP];
            cheb4(P, (pxT[pos] - cx) * irx, Sx);
            cheb4(P, (pyT[pos] - cy) * iry, Sy);
            f32x4 a;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = 4 * h + e;
                a[e] = p < cnt ? (float)(Sx[k & 3] * Sy[k >> 2]) : 0.f;
            }
            acc = mfma16(a, loc, acc);
        }
        const f32x4* kt = Knear + koff[w] + (size_t)rb * nst4 * 64 + lane;
        for (int s4 = 0; s4 < nst4; ++s4) {
            const f32x4 a = __builtin_nontemporal_load(kt + (size_t)s4 * 64);
            f32x4 f;
#pragma unroll
            for (int e = 0; e < 4; ++e) f[e] = fT[(size_t)nearPts[pb + 16 * s4 + 4 * e + h] * 16 + r];
            acc = mfma16(a, f, acc);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // lane: points 16 rb + 4h + e, right-hand side r
            const int p = 16 * rb + 4 * h + e;
            if (p < cnt) {
                const int64_t pos = b + p;
                Y[pos * 16 + r] = X[pos * 16 + r] - scale * acc[e];
            }
        }
    }
}

// fp64 column-major M2L blocks (k_cache_m2l: pair*256 + s*16 + t) -> fp32 A order
// (lane l, element e = K[t = l&15][s = 4(l>>4) + e])
__global__ void k32_conv_m2l(int64_t n, const double* __restrict__ Kd, float* __restrict__ K32) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n * 256) return;
    const int64_t p = id >> 8;
    const int l = (int)((id >> 2) & 63), e = (int)(id & 3);
    K32[id] = (float)Kd[p * 256 + (4 * (l >> 4) + e) * 16 + (l & 15)];
}

// fp64 near blocks of one chunk of leaves (k_cache_near: nT4 x S column-major, rows
// padded to 4) -> fp32 tiles (k32_leaf); one thread per tile float
__global__ void k32_conv_near(int nl, const int4* __restrict__ info, const int64_t* __restrict__ koffD,
                              const int64_t* __restrict__ koff, const int* __restrict__ srcCount,
                              const double* __restrict__ Kd, float* __restrict__ K32) {
    const int li = blockIdx.y;
    if (li >= nl) return;
    const int4 in = info[li];
    const int nT = in.z, Sp = in.w, S = srcCount[li];
    const int nT4 = (nT + 3) & ~3, nrb = (nT + 15) >> 4, nst4 = Sp >> 4;
    const int64_t total = (int64_t)nrb * nst4 * 256;
    float* dst = K32 + koff[li] * 4;
    const double* src = Kd + koffD[li];
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(id & 3), l = (int)((id >> 2) & 63);
        const int64_t tile = id >> 8;
        const int s4 = (int)(tile % nst4), rb = (int)(tile / nst4);
        const int t = 16 * rb + (l & 15), s = 16 * s4 + 4 * e + (l >> 4);
        dst[id] = (t < nT && s < S) ? (float)src[(int64_t)s * nT4 + t] : 0.f;
    }
}

// ----------------------------------------------------------------- launchers

void launch32_p2m(int nleaf, const int* leaves, const int64_t* begin, const int64_t* count, const double* ncx,
                  const double* ncy, const double* nrx, const double* nry, const double* pxT, const double* pyT,
                  const float* X, const double* sigT, const double* wT, const Params* P, void* mult, float* fT,
                  float* cT, hipStream_t s) {
    if (nleaf <= 0) return;
    k32_p2m<<<blocks_for((int64_t)nleaf * kWave, 256), 256, 0, s>>>(nleaf, leaves, begin, count, ncx, ncy, nrx, nry,
                                                                   pxT, pyT, X, sigT, wT, P,
                                                                   static_cast<f32x4*>(mult), fT, cT);
    HIP_LAUNCH_CHECK();
}

void launch32_m2m(int nn, const int* nodes, const int4* child, const int64_t* count, const void* Rup, void* mult,
                  hipStream_t s) {
    if (nn <= 0) return;
    k32_m2m<<<blocks_for((int64_t)nn * kWave, 256), 256, 0, s>>>(nn, nodes, child, count,
                                                                static_cast<const f32x4*>(Rup),
                                                                static_cast<f32x4*>(mult));
    HIP_LAUNCH_CHECK();
}

void launch32_m2l(int ntgt, const int* tgt, const int64_t* ptr, const int* src, const void* K32, const void* mult,
                  void* local, hipStream_t s) {
    if (ntgt <= 0) return;
    k32_m2l<<<blocks_for((int64_t)ntgt * kWave, 256), 256, 0, s>>>(ntgt, tgt, ptr, src, static_cast<const f32x4*>(K32),
                                                                  static_cast<const f32x4*>(mult),
                                                                  static_cast<f32x4*>(local));
    HIP_LAUNCH_CHECK();
}

void launch32_l2l(int nn, const int* nodes, const int* parent, const int* slot, const void* Rdn, void* local,
                  hipStream_t s) {
    if (nn <= 0) return;
    k32_l2l<<<blocks_for((int64_t)nn * kWave, 256), 256, 0, s>>>(nn, nodes, parent, slot,
                                                                static_cast<const f32x4*>(Rdn),
                                                                static_cast<f32x4*>(local));
    HIP_LAUNCH_CHECK();
}

void launch32_leaf(int nleaf, const int4* leafInfo, const int64_t* nearPtr, const int* nearPts, const int64_t* koff,
                   const void* Knear, const int* level, const double* ncx, const double* ncy, const double* nrx,
                   const double* nry, const double* pxT, const double* pyT, const Params* P, const void* local,
                   const float* fT, const float* X, float scale, int flags, float* Y, hipStream_t s) {
    if (nleaf <= 0) return;
    k32_leaf<<<blocks_for((int64_t)nleaf * kWave, 256), 256, 0, s>>>(
        nleaf, leafInfo, nearPtr, nearPts, koff, static_cast<const f32x4*>(Knear), level, ncx, ncy, nrx, nry, pxT,
        pyT, P, static_cast<const f32x4*>(local), fT, X, scale, flags, Y);
    HIP_LAUNCH_CHECK();
}

void launch32_corr(int d, int64_t N, const int* perm, const int* iperm, const float* cT, const float* fT,
                   const double* C, const double* mu, const Params* P, int flags, float scale, float* Y,
                   hipStream_t s) {
    if (N <= 0) return;
    const unsigned nb = blocks_for(N, 256);
    switch (d) {
        case 1: k16_corr<float, 1><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 2: k16_corr<float, 2><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 3: k16_corr<float, 3><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 4: k16_corr<float, 4><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 5: k16_corr<float, 5><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        case 6: k16_corr<float, 6><<<nb, 256, 0, s>>>(N, perm, iperm, cT, fT, C, mu, P, flags, scale, Y); break;
        default: throw std::invalid_argument("quadRule out of range");
    }
    HIP_LAUNCH_CHECK();
}

void launch32_conv_m2l(int64_t npairs, const double* Kd, void* K32, hipStream_t s) {
    if (npairs <= 0) return;
    k32_conv_m2l<<<blocks_for(npairs * 256, 256), 256, 0, s>>>(npairs, Kd, static_cast<float*>(K32));
    HIP_LAUNCH_CHECK();
}

void launch32_conv_near(int nl, const int4* info, const int64_t* koffD, const int64_t* koff, const int* srcCount,
                        const double* Kd, void* K32, hipStream_t s) {
    if (nl <= 0) return;
    dim3 grid(4, (unsigned)nl);
    k32_conv_near<<<grid, 256, 0, s>>>(nl, info, koffD, koff, srcCount, Kd, static_cast<float*>(K32));
    HIP_LAUNCH_CHECK();
}

}  // namespace aniso
