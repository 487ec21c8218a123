// m2l_micro.hip -- isolates what bounds the M2L operator stream (not part of the
// product).  Synthetic plan shaped like the 1M-point uniform tree: T targets,
// per-target pair counts drawn to match, random sources; times
//   dir27  : k_m2l, 27 directed pairs per target
//   dir13  : k_m2l, 13-14 directed pairs per target (same bytes as canonical)
//   can13  : k_m2l, 13-14 canonical pairs per target (transposed products stored)
//   canvar : k_m2l, canonical counts 0..27 (uniform-tree-like spread)
//   copy   : a plain float4 stream of the same byte count
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/m2l_micro.hip -o /tmp/m2l_micro
#include "../aniso_amd/csrc/kernels.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace aniso;

namespace aniso {
[[noreturn]] void throw_hip(hipError_t e, const char* file, int line) {
    std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), file, line);
    std::exit(1);
}
}  // namespace aniso

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

__global__ void k_copy(const dbl2* __restrict__ a, int64_t n, double* __restrict__ out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        dbl2 v = __builtin_nontemporal_load(a + i);
        s += v.x + v.y;
    }
    if (s == 12345.678) out[0] = s;
}


// experiment copies of k_m2l's canonical section: STORE 0 none, 1 receiver slots
// (product), 2 sender-contiguous; TR 0 skips the transposed product
template <int STORE, int TR, int PERSIST>
__global__ void __launch_bounds__(256) k_can(int ntgt, const int64_t* __restrict__ ptr, const int* __restrict__ canonBase,
                                             const int* __restrict__ outSlot, const int* __restrict__ src,
                                             const double* __restrict__ K, const double* __restrict__ mult,
                                             double* __restrict__ partial, double* __restrict__ local) {
    const int wave0 = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) / kWave));
    const int lane = threadIdx.x & (kWave - 1);
    const int nw = PERSIST ? (int)(gridDim.x * blockDim.x / kWave) : 1;
    for (int wave = wave0; wave < ntgt; wave += nw) {
    if (!PERSIST && wave != wave0) break;
    const int n = wave;
    const int t = lane >> 2, q = lane & 3;
    const int64_t pd = ptr[wave], p1 = ptr[wave + 1];
    const int nC = (int)(p1 - pd);
    const int cSrc = lane < nC ? src[pd + lane] : 0;
    const int cSlot = lane < nC ? outSlot[canonBase[wave] + lane] : 0;
    double acc = 0.0;
    if (nC > 0) {
        const double4 mn = *reinterpret_cast<const double4*>(mult + (size_t)n * kRank + q * 4);
        const double m0 = mn.x, m1 = mn.y, m2 = mn.z, m3 = mn.w;
        double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
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
                if (TR) {
                    const double ya = quad_sum(a0.x * m0 + a0.y * m1 + a1.x * m2 + a1.y * m3);
                    const double yb = quad_sum(b0.x * m0 + b0.y * m1 + b1.x * m2 + b1.y * m3);
                    const double ye = quad_sum(e0.x * m0 + e0.y * m1 + e1.x * m2 + e1.y * m3);
                    const double yf = quad_sum(f0.x * m0 + f0.y * m1 + f1.x * m2 + f1.y * m3);
                    y[g] = q == 0 ? ya : q == 1 ? yb : q == 2 ? ye : yf;
                }
            }
        }
        if (STORE) {
#pragma unroll
            for (int g = 0; g < kGroups; ++g) {
                if (4 * g < nC) {
                    const int jj = 4 * g + q;
                    int slot = STORE != 2 ? __shfl(cSlot, jj) : canonBase[wave] + jj;
                    if (STORE == 6) slot &= 1023;  // L2-resident footprint (128 KB)
                    if (STORE == 7) slot &= (1 << 15) - 1;  // 4 MB
                    if (STORE == 8) slot &= (1 << 18) - 1;  // 32 MB
                    if (STORE == 9) slot &= (1 << 19) - 1;  // 64 MB
                    if (jj < nC && (STORE != 5 || jj % 3 == 0)) {
                        if (STORE == 3)
                            __builtin_nontemporal_store(y[g], partial + (size_t)slot * kRank + t);
                        else if (STORE == 4)
                            __hip_atomic_store(partial + (size_t)slot * kRank + t, y[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        else
                            partial[(size_t)slot * kRank + t] = y[g];
                    }
                }
            }
        } else {
            double z = 0.0;
            for (int g = 0; g < kGroups; ++g) z += y[g];
            acc += z;
        }
#pragma unroll
        for (int off = 4; off < kWave; off <<= 1) {
            c0 += __shfl_xor(c0, off);
            c1 += __shfl_xor(c1, off);
            c2 += __shfl_xor(c2, off);
            c3 += __shfl_xor(c3, off);
        }
        const int jr = t & 3;
        const double v = jr == 0 ? c0 : jr == 1 ? c1 : jr == 2 ? c2 : c3;
        const double w = __shfl(v, 4 * t + (t >> 2));
        if (q == 0) acc += w;
    }
    acc = quad_sum(acc);
    if (q == 0) local[(size_t)n * kRank + t] = acc;
    }
}

// persistent waves; the partial stores of target i are issued after the first
// operator loads of target i+1 so no wait on the loads waits on the stores
__global__ void __launch_bounds__(256) k_can_pipe(int ntgt, const int64_t* __restrict__ ptr, const int* __restrict__ canonBase,
                                                  const int* __restrict__ outSlot, const int* __restrict__ src,
                                                  const double* __restrict__ K, const double* __restrict__ mult,
                                                  double* __restrict__ partial, double* __restrict__ local) {
    const int wave0 = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) / kWave));
    const int lane = threadIdx.x & (kWave - 1);
    const int nw = (int)(gridDim.x * blockDim.x / kWave);
    const int t = lane >> 2, q = lane & 3;
    constexpr int kGroups = (kMaxCanon + 3) / 4;
    double yp[kGroups];
    int slotp[kGroups];
    int nCp = 0;
    for (int wave = wave0; wave < ntgt + nw; wave += nw) {
        const bool live = wave < ntgt;
        const int n = wave;
        const int64_t pd = live ? ptr[wave] : 0, p1 = live ? ptr[wave + 1] : 0;
        const int nC = (int)(p1 - pd);
        const int cSrc = lane < nC ? src[pd + lane] : 0;
        const int cSlot = lane < nC ? outSlot[canonBase[live ? wave : 0] + lane] : 0;
        // first group's loads
        dbl2 a0, a1, b0, b1, e0, e1, f0, f1;
        load_block(K, pd, lane, nC > 0, a0, a1);
        load_block(K, pd + 1, lane, nC > 1, b0, b1);
        load_block(K, pd + 2, lane, nC > 2, e0, e1);
        load_block(K, pd + 3, lane, nC > 3, f0, f1);
        // previous target's partials
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
            if (4 * g < nCp) {
                const int jj = 4 * g + q;
                if (jj < nCp) partial[(size_t)slotp[g] * kRank + t] = yp[g];
            }
        }
        if (!live) break;
        const double4 mn = *reinterpret_cast<const double4*>(mult + (size_t)n * kRank + q * 4);
        const double m0 = mn.x, m1 = mn.y, m2 = mn.z, m3 = mn.w;
        double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
            yp[g] = 0.0;
            const int j = 4 * g;
            if (j < nC) {
                if (g > 0) {
                    load_block(K, pd + j, lane, true, a0, a1);
                    load_block(K, pd + j + 1, lane, j + 1 < nC, b0, b1);
                    load_block(K, pd + j + 2, lane, j + 2 < nC, e0, e1);
                    load_block(K, pd + j + 3, lane, j + 3 < nC, f0, f1);
                }
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
                yp[g] = q == 0 ? ya : q == 1 ? yb : q == 2 ? ye : yf;
                slotp[g] = __shfl(cSlot, (4 * g + q) & 63);
            }
        }
        nCp = nC;
#pragma unroll
        for (int off = 4; off < kWave; off <<= 1) {
            c0 += __shfl_xor(c0, off);
            c1 += __shfl_xor(c1, off);
            c2 += __shfl_xor(c2, off);
            c3 += __shfl_xor(c3, off);
        }
        const int jr = t & 3;
        const double v = jr == 0 ? c0 : jr == 1 ? c1 : jr == 2 ? c2 : c3;
        double acc = __shfl(v, 4 * t + (t >> 2));
        if (q == 0) local[(size_t)n * kRank + t] = acc;
    }
}

struct Case {
    const char* name;
    std::vector<int> nDir, nCan;
};

int main() {
    const int T = 87380, NN = 87381;
    std::mt19937 rng(1);
    std::vector<Case> cases;
    {
        Case c{"dir27", {}, {}};
        for (int i = 0; i < T; ++i) { c.nDir.push_back(27); c.nCan.push_back(0); }
        cases.push_back(c);
    }
    {
        Case c{"dir13", {}, {}};
        for (int i = 0; i < T; ++i) { c.nDir.push_back(13 + (i & 1)); c.nCan.push_back(0); }
        cases.push_back(c);
    }
    {
        Case c{"can13", {}, {}};
        for (int i = 0; i < T; ++i) { c.nDir.push_back(0); c.nCan.push_back(13 + (i & 1)); }
        cases.push_back(c);
    }
    {
        Case c{"canvar", {}, {}};
        std::uniform_int_distribution<int> u(0, 27);
        for (int i = 0; i < T; ++i) { c.nDir.push_back(0); c.nCan.push_back(u(rng)); }
        cases.push_back(c);
    }
    int64_t maxPairs = (int64_t)T * 27;
    double *K, *mult, *local, *partial, *dummy;
    CK(hipMalloc(&K, maxPairs * 256 * sizeof(double)));
    CK(hipMemset(K, 0, maxPairs * 256 * sizeof(double)));
    CK(hipMalloc(&mult, (size_t)NN * 16 * sizeof(double)));
    CK(hipMemset(mult, 0, (size_t)NN * 16 * sizeof(double)));
    CK(hipMalloc(&local, (size_t)NN * 16 * sizeof(double)));
    CK(hipMalloc(&partial, maxPairs * 16 * sizeof(double)));
    CK(hipMalloc(&dummy, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::uniform_int_distribution<int> us(0, NN - 1);
    for (auto& c : cases) {
        std::vector<int> tgt(T), nDir(T), cbase(T), src;
        std::vector<int64_t> ptr(T + 1, 0);
        int canon = 0;
        for (int i = 0; i < T; ++i) {
            tgt[i] = i;
            nDir[i] = c.nDir[i];
            cbase[i] = canon;
            for (int k = 0; k < c.nDir[i] + c.nCan[i]; ++k) src.push_back(us(rng));
            canon += c.nCan[i];
            ptr[i + 1] = (int64_t)src.size();
        }
        std::vector<int> slot(canon);
        for (int k = 0; k < canon; ++k) slot[k] = k;
        std::shuffle(slot.begin(), slot.end(), rng);
        int *dT, *dD, *dB, *dS, *dSl;
        int64_t* dP;
        CK(hipMalloc(&dT, T * 4)); CK(hipMemcpy(dT, tgt.data(), T * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&dD, T * 4)); CK(hipMemcpy(dD, nDir.data(), T * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&dB, T * 4)); CK(hipMemcpy(dB, cbase.data(), T * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&dS, src.size() * 4)); CK(hipMemcpy(dS, src.data(), src.size() * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&dSl, std::max(canon, 1) * 4));
        if (canon) CK(hipMemcpy(dSl, slot.data(), canon * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&dP, (T + 1) * 8)); CK(hipMemcpy(dP, ptr.data(), (T + 1) * 8, hipMemcpyHostToDevice));
        const int reps = 20;
        for (int w = 0; w < 3; ++w) launch_m2l(T, dT, dP, dD, dB, dSl, dS, K, mult, 1.0, partial, local, 0);
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch_m2l(T, dT, dP, dD, dB, dSl, dS, K, mult, 1.0, partial, local, 0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        double bytes = 2048.0 * src.size() + 256.0 * T + 128.0 * canon;
        std::printf("%-8s pairs %9zu  %.4f ms  %.1f GB/s\n", c.name, src.size(), ms, bytes / ms / 1e6);
        if (canon && c.nDir[0] == 0) {
            auto run = [&](const char* nm, auto kern, int grid = (T * 64 + 255) / 256) {
                for (int w = 0; w < 3; ++w) kern<<<grid, 256>>>(T, dP, dB, dSl, dS, K, mult, partial, local);
                CK(hipEventRecord(e0, 0));
                for (int r = 0; r < reps; ++r) kern<<<grid, 256>>>(T, dP, dB, dSl, dS, K, mult, partial, local);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float m = 0;
                CK(hipEventElapsedTime(&m, e0, e1));
                m /= reps;
                std::printf("%-8s %-14s %.4f ms  %.1f GB/s (operator bytes only)\n", c.name, nm, m, 2048.0 * src.size() / m / 1e6);
            };
            run("store=slot", k_can<1, 1, 0>);
            run("store=contig", k_can<2, 1, 0>);
            run("store=none", k_can<0, 1, 0>);
            run("no-transpose", k_can<0, 0, 0>);
            run("store=1/3", k_can<5, 1, 0>);
            run("store=l2", k_can<6, 1, 0>);
            run("store=4MB", k_can<7, 1, 0>);
            run("store=32MB", k_can<8, 1, 0>);
            run("store=64MB", k_can<9, 1, 0>);
            for (int wpc : std::initializer_list<int>{}) {
                char nm[64];
                std::snprintf(nm, sizeof nm, "pipe%d", wpc);
                run(nm, k_can_pipe, 256 * wpc / 4);
            }
            run("store=nt", k_can<3, 1, 0>);
            run("store=sys", k_can<4, 1, 0>);
            for (int wpc : std::initializer_list<int>{}) {
                char nm[64];
                std::snprintf(nm, sizeof nm, "persist%d/slot", wpc);
                run(nm, k_can<1, 1, 1>, 256 * wpc / 4);
                std::snprintf(nm, sizeof nm, "persist%d/none", wpc);
                run(nm, k_can<0, 1, 1>, 256 * wpc / 4);
            }
        }
        // the same bytes as a plain stream
        int64_t n4 = (int64_t)src.size() * 2048 / 16;
        for (int w = 0; w < 2; ++w) k_copy<<<4096, 256>>>(reinterpret_cast<const dbl2*>(K), n4, dummy);
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) k_copy<<<4096, 256>>>(reinterpret_cast<const dbl2*>(K), n4, dummy);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        std::printf("%-8s copy  %.4f ms  %.1f GB/s\n", c.name, ms, n4 * 16.0 / ms / 1e6);
        hipFree(dT); hipFree(dD); hipFree(dB); hipFree(dS); hipFree(dSl); hipFree(dP);
    }
    return 0;
}
