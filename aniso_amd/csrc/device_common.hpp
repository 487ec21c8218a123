// device_common.hpp -- device helpers shared by the apply kernels (apply.hip) and
// the cache-build kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace aniso {

[[noreturn]] void throw_hip(hipError_t e, const char* file, int line);

#define HIP_LAUNCH_CHECK()                                                                  \
    do {                                                                                    \
        hipError_t e__ = hipGetLastError();                                                 \
        if (e__ != hipSuccess) throw_hip(e__, __FILE__, __LINE__);                          \
    } while (0)

constexpr int kWave = 64;
typedef double dbl2 __attribute__((ext_vector_type(2)));

static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

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

// Lane-quad exchange through DPP quad_perm (no LDS round trip).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
// v of lane (lane ^ OFF) within a 16-lane DPP row, OFF in {1, 2, 4, 8}, on the VALU
// (no LDS permute): quad_perm for 1 and 2, row_ror:8 for 8; for 4 it is row_ror:4
// on half of the lanes and row_ror:12 on the other half -- r4 (from
// xor16_r4(lane)) says which, measured from the hardware's own lane ids, so the
// rotate direction is not assumed.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ bool xor16_r4(int lane) {
    const int ln = lane & 15;
    return dpp_i32<0x124>(ln) == (ln ^ 4);
}
template <int OFF>
__device__ __forceinline__ double xor16_f64(double v, bool r4) {
    if constexpr (OFF == 1) return dpp_f64<0xB1>(v);
    else if constexpr (OFF == 2) return dpp_f64<0x4E>(v);
    else if constexpr (OFF == 8) return dpp_f64<0x128>(v);
    else {
        static_assert(OFF == 4, "xor16_f64: OFF in {1, 2, 4, 8}");
        const double a = dpp_f64<0x124>(v), b = dpp_f64<0x12C>(v);
        return r4 ? a : b;
    }
}

// Reduce-scatter steps across lane ^ 16 / lane ^ 32 (gfx950 v_permlane16/32_swap with
// x in VDST and y in SRC0): one lane of each pair ends with x + x', the other with
// y + y' -- which one is measured by the caller (probe with x = 1, y = 0), not assumed.
__device__ __forceinline__ double swap_add16_f64(double x, double y) {
    const unsigned long long bx = __builtin_bit_cast(unsigned long long, x), by = __builtin_bit_cast(unsigned long long, y);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)bx, (unsigned)by, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(bx >> 32), (unsigned)(by >> 32), false, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]) +
           __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double swap_add32_f64(double x, double y) {
    const unsigned long long bx = __builtin_bit_cast(unsigned long long, x), by = __builtin_bit_cast(unsigned long long, y);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)bx, (unsigned)by, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(bx >> 32), (unsigned)(by >> 32), false, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]) +
           __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
}

// v(lane) + v(lane ^ 16) and v(lane) + v(lane ^ 32) through gfx950's
// v_permlane16/32_swap (row exchange on the VALU; the sum of both swap outputs is
// the pair sum whichever row each output holds).
__device__ __forceinline__ double xsum16_f64(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    const double a = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
    const double c = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
    return a + c;
}
__device__ __forceinline__ double xsum32_f64(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    const double a = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
    const double c = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
    return a + c;
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

// Row stride of the tree-order charge arrays fT/cT [N][KS]: K rounded up to even
// (K > 1) so a row is whole 16-B vectors.
template <int K>
constexpr int kStride = (K == 1 || K % 2 == 0) ? K : K + 1;

// Output slot of tree position k: the original index perm[k] (original-order
// output) or the owned tree-order slice k - obase (operm == nullptr).
__device__ __forceinline__ int64_t out_index(const int* __restrict__ operm, int64_t obase, int64_t k) {
    return operm ? (int64_t)operm[k] : k - obase;
}

// Store the K charges of one tree position as whole 16-B vectors (the pad entry of
// an odd K is written as 0): one lane's row is contiguous, so a wave's consecutive
// points write whole lines instead of K strided 8-B stores.
template <int K>
__device__ __forceinline__ void store_charges(double* __restrict__ p, const double (&c)[K]) {
    if constexpr (K == 1) {
        p[0] = c[0];
    } else {
#pragma unroll
        for (int v = 0; v < kStride<K> / 2; ++v)
            reinterpret_cast<dbl2*>(p)[v] = dbl2{c[2 * v], 2 * v + 1 < K ? c[2 * v + 1] : 0.0};
    }
}

// Load the K charges of one tree position (row of fT / cT, stride kStride<K>).
template <int K>
__device__ __forceinline__ void load_charges(const double* __restrict__ p, double (&c)[K]) {
    if constexpr (K == 1) {
        c[0] = p[0];
    } else {
#pragma unroll
        for (int v = 0; v < kStride<K> / 2; ++v) {
            const dbl2 x = reinterpret_cast<const dbl2*>(p)[v];
            c[2 * v] = x.x;
            if (2 * v + 1 < K) c[2 * v + 1] = x.y;
        }
    }
}

}  // namespace aniso
