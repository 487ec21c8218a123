// arnoldi_micro.hip -- bandwidth of the DCGS2 sweeps (aniso_amd/csrc/arnoldi.hpp) at the
// block solve's vector length (5 x 1M doubles), against a plain 16-B copy; not part of
// the product.  For nv basis rows: sweep A reads nv + 1 vectors, sweep B reads nv + 1
// and writes 1; then the small kernels.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I aniso_amd/csrc tools/arnoldi_micro.hip -o tools/arnoldi_micro.bin
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "arnoldi.hpp"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

using namespace aniso;
typedef double d2v __attribute__((ext_vector_type(2)));

__global__ void k_copy2(int64_t n, const d2v* __restrict__ a, d2v* __restrict__ b) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__global__ void k_fill(int64_t n, double* v, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        v[i] = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
}

// layout experiment: the basis tiled as [tile][row][TE elements] (a tile's rows contiguous)
template <int NV, int TE>
__global__ void __launch_bounds__(256) k_project_tiled(int64_t ntiles, int nv, int m1, const double* __restrict__ Vt,
                                                       const double* __restrict__ w, double* __restrict__ part) {
    __shared__ double red[4 * NV];
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    const int64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    const int64_t t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
    for (int64_t t = t0; t < t1; ++t)
        for (int e = threadIdx.x; e < TE; e += 256) {
            const double* base = Vt + (size_t)t * m1 * TE + e;
            double v[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k)
                if (k < nv) v[k] = base[(size_t)k * TE];
            const double we = w[t * TE + e];
#pragma unroll
            for (int k = 0; k < NV; ++k)
                if (k < nv) acc[k] = __builtin_fma(v[k], we, acc[k]);
        }
    arn::block_store<NV>(acc, nv, -1, red, part, blockIdx.x);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 5 * 1048576;
    const int maxv = 60;
    double *V, *w, *part, *st, *V2;
    CK(hipMalloc(&V, (size_t)maxv * n * sizeof(double)));
    CK(hipMalloc(&V2, (size_t)maxv * n * sizeof(double)));
    CK(hipMalloc(&w, n * sizeof(double)));
    CK(hipMalloc(&part, (size_t)4096 * (maxv + 2) * sizeof(double)));
    const int m = 64;
    arn::Layout L(m);
    CK(hipMalloc(&st, L.total * sizeof(double)));
    k_fill<<<2048, 256>>>((int64_t)maxv * n, V, 1);
    k_fill<<<2048, 256>>>(n, w, 2);
    k_fill<<<2048, 256>>>(L.total, st, 3);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double vecGB = n * 8.0 / 1e9;
    auto time = [&](auto&& f, int reps) {
        f();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    {
        const float ms = time([&] { k_copy2<<<4096, 256>>>(n, (const d2v*)V, (d2v*)V2); }, 20);
        std::printf("copy16 %.4f ms %.1f GB/s\n", ms, 2 * vecGB / (ms * 1e-3));
    }
    std::vector<double> h(4096 * (maxv + 2));
    for (int nv : {4, 8, 16, 24, 32, 40, 48, 56}) {
        const float ms = time([&] { arn::launch_project(n, nv, V, n, w, part, 0); }, 10);
        std::printf("project nv %2d: %.4f ms %.1f GB/s\n", nv, ms, (nv + 1) * vecGB / (ms * 1e-3));
    }
    auto var = [&](auto vc, const char* name) {
        constexpr int VAR = decltype(vc)::value;
        for (int nv : {8, 16, 24, 32, 48}) {
            CK(hipMemcpy(V2, V, (size_t)(nv + 1) * n * sizeof(double), hipMemcpyDeviceToDevice));
            const float ms = time([&] { arn::launch_update<VAR>(n, nv, V2, n, w, st, m, part, 0); }, 10);
            std::printf("update %-8s nv %2d: %.4f ms %.1f GB/s (reads %d vectors)\n", name, nv, ms,
                        (nv + 2) * vecGB / (ms * 1e-3), nv + 1);
        }
    };
    var(std::integral_constant<int, 0>{}, "base");
    var(std::integral_constant<int, 1>{}, "reverse");
    var(std::integral_constant<int, 4>{}, "nt");
    for (int64_t pad : {256, 576, 4224, 65536 + 192}) {
        const int64_t ld = n + pad;
        for (int nv : {8, 24, 48}) {
            const float ma = time([&] { arn::launch_project(n, nv, V2, ld, w, part, 0); }, 10);
            const float mb = time([&] { arn::launch_update(n, nv, V2, ld, w, st, m, part, 0); }, 10);
            std::printf("pad %6lld nv %2d: project %.4f ms %.1f GB/s  update %.4f ms %.1f GB/s\n", (long long)pad, nv,
                        ma, (nv + 1) * vecGB / (ma * 1e-3), mb, (nv + 2) * vecGB / (mb * 1e-3));
        }
    }
    // the small kernels on kParts partials
    (void)hipFuncSetAttribute((const void*)arn::k_arn_coef, hipFuncAttributeMaxDynamicSharedMemorySize, 136 * 1024);
    (void)hipFuncSetAttribute((const void*)arn::k_arn_column, hipFuncAttributeMaxDynamicSharedMemorySize, 136 * 1024);
    for (int j : {0, 15, 39, 63}) {
        k_fill<<<2048, 256>>>(L.total, st, 3);
        const float mc = time([&] { arn::k_arn_coef<<<1, 256, arn::coef_lds(j)>>>(m, j, st, part, arn::kParts); }, 20);
        const float mk = time([&] {
            arn::k_arn_column<<<1, 256, arn::column_lds(j)>>>(m, j, st, part, arn::kParts, nullptr);
        }, 20);
        const float mr = time([&] {
            arn::k_arn_rows<<<1, 256, (j + 2) * sizeof(double)>>>(part, arn::kParts, j + 2, w);
        }, 20);
        std::printf("coef j %2d: %.2f us  column: %.2f us  rows: %.2f us\n", j, mc * 1e3, mk * 1e3, mr * 1e3);
    }
    {
        const float ms = time([&] { arn::k_arn_solve<<<1, 256, arn::solve_lds(40)>>>(m, 40, st); }, 20);
        std::printf("solve used 40: %.2f us\n", ms * 1e3);
    }
    CK(hipDeviceSynchronize());
    std::printf("done\n");
    return 0;
}
