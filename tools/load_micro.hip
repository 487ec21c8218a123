// load_micro.hip -- what the per-lane load shape of the E stream costs (not part of
// the product).  Streams NB 2-KB blocks (one block per wave step, like the M2L)
// with different lane -> address maps and reports GB/s of block bytes:
//   frag  : lane l loads 16 B at 32 l and 32 l + 16 (k_m2l_hc's stored orientation:
//           each instruction touches 16 lines, 64 B of each)
//   line  : lane l loads 16 B at 16 l and 1024 + 16 l (each instruction: 8 full lines)
//   tr    : four 8-B loads at 8 (64 q + s + 16 j) (the transposed orientation)
//   fragm : frag + three mult-like loads per block (40 B per lane, 4 lanes share an
//           address, random node of a 56 MB table)
//   linem : line + the same mult-like loads
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/load_micro.hip -o /tmp/load_micro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

struct dbl2 {
    double x, y;
};

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

template <int MODE, bool MULT, int PG>
__global__ void __launch_bounds__(256) k_stream(int64_t nb, int steps, const double* __restrict__ E,
                                                const double* __restrict__ mult, int nnode,
                                                double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int s = lane >> 2, q = lane & 3;
    double acc = 0.0;
    for (int it = 0; it < steps; it += PG) {
        double v[PG][4];
        double m[PG][5];
#pragma unroll
        for (int g = 0; g < PG; ++g) {
            const int64_t b = (wave * steps + it + g) % nb;
            const double* p = E + b * 256;
            if (MODE == 0) {
                const dbl2* d = reinterpret_cast<const dbl2*>(p + 4 * lane);
                const dbl2 a = d[0], c = d[1];
                v[g][0] = a.x; v[g][1] = a.y; v[g][2] = c.x; v[g][3] = c.y;
            } else if (MODE == 1) {
                const dbl2 a = reinterpret_cast<const dbl2*>(p)[lane];
                const dbl2 c = reinterpret_cast<const dbl2*>(p + 128)[lane];
                v[g][0] = a.x; v[g][1] = a.y; v[g][2] = c.x; v[g][3] = c.y;
            } else {
                const double* t = p + 64 * q + s;
#pragma unroll
                for (int j = 0; j < 4; ++j) v[g][j] = t[16 * j];
            }
            if (MULT) {
                const int B = (int)((b * 2654435761u) % (uint64_t)nnode);
                const double* mm = mult + ((size_t)B * 16 + s) * 5;
#pragma unroll
                for (int k = 0; k < 5; ++k) m[g][k] = mm[k];
            }
        }
#pragma unroll
        for (int g = 0; g < PG; ++g) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += v[g][j];
            if (MULT)
#pragma unroll
                for (int k = 0; k < 5; ++k) acc += m[g][k];
        }
    }
    if (acc == 1234.5) out[0] = acc;
}


// the M2L's per-entry arithmetic (harmonic.hip hm_entry, K = 5, one Newton step) on
// the streamed blocks: PF = 1 issues the next group's loads before this group's math
__device__ __forceinline__ void entry5(double e, double dx, double dy2, const double (&xw)[5], double (&o)[5]) {
    const double r2 = __builtin_fma(dx, dx, dy2);
    const double y = __builtin_amdgcn_rsq(r2);
    const double ri = __builtin_fma(0.5 * y, __builtin_fma(-(r2 * y), y, 1.0), y);
    const double c = dx * ri;
    double T[5];
    T[0] = 1.0; T[1] = c;
    const double c2 = c + c;
#pragma unroll
    for (int i = 2; i < 5; ++i) T[i] = __builtin_fma(c2, T[i - 1], -T[i - 2]);
    double v = xw[0];
#pragma unroll
    for (int b = 1; b < 5; ++b) v = __builtin_fma(T[b], xw[b], v);
    const double av = (e * ri) * v;
#pragma unroll
    for (int i = 0; i < 5; ++i) o[i] = __builtin_fma(T[i], av, o[i]);
}

template <int PG, bool PF, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
k_m2l_like(int64_t nb, int steps, const double* __restrict__ E, const double* __restrict__ mult, int nnode,
           double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int s = lane >> 2, q = lane & 3;
    double o[4][5];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 5; ++i) o[j][i] = 0.0;
    const double bx0 = 0.1 * q, by = 0.01 * s;
    double v[PG][4], m[PG][5];
    auto load = [&](int it) {
#pragma unroll
        for (int g = 0; g < PG; ++g) {
            const int64_t b = (wave * steps + it + g) % nb;
            const dbl2* d = reinterpret_cast<const dbl2*>(E + b * 256 + 4 * lane);
            const dbl2 a = d[0], c = d[1];
            v[g][0] = a.x; v[g][1] = a.y; v[g][2] = c.x; v[g][3] = c.y;
            const int B = (int)((b * 2654435761u) % (uint64_t)nnode);
            const double* mm = mult + ((size_t)B * 16 + s) * 5;
#pragma unroll
            for (int k = 0; k < 5; ++k) m[g][k] = mm[k];
        }
    };
    if (PF) load(0);
    for (int it = 0; it < steps; it += PG) {
        double cv[PG][4], cm[PG][5];
        if (PF) {
#pragma unroll
            for (int g = 0; g < PG; ++g) {
#pragma unroll
                for (int j = 0; j < 4; ++j) cv[g][j] = v[g][j];
#pragma unroll
                for (int k = 0; k < 5; ++k) cm[g][k] = m[g][k];
            }
            if (it + PG < steps) load(it + PG);
        } else {
            load(it);
#pragma unroll
            for (int g = 0; g < PG; ++g) {
#pragma unroll
                for (int j = 0; j < 4; ++j) cv[g][j] = v[g][j];
#pragma unroll
                for (int k = 0; k < 5; ++k) cm[g][k] = m[g][k];
            }
        }
#pragma unroll
        for (int g = 0; g < PG; ++g) {
            const double ax = 0.3 + 0.001 * (it + g) + 0.02 * s, dy = by - 0.2 * q - 0.5;
            double xw[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) xw[k] = 0.7 * cm[g][k];
#pragma unroll
            for (int j = 0; j < 4; ++j) entry5(cv[g][j], ax - bx0 - 0.05 * j, dy * dy, xw, o[j]);
        }
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 5; ++i) acc += o[j][i];
    if (acc == 1234.5) out[0] = acc;
}

template <int PG, bool PF, int WPE>
double run_c(int64_t nb, const double* E, const double* mult, int nnode, double* out) {
    const int steps = 32;
    const int64_t waves = nb / steps;
    const int grid = (int)((waves * 64 + 255) / 256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_m2l_like<PG, PF, WPE><<<grid, 256>>>(nb, steps, E, mult, nnode, out);
    CK(hipEventRecord(a));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) k_m2l_like<PG, PF, WPE><<<grid, 256>>>(nb, steps, E, mult, nnode, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;  // ms per launch
}

template <int MODE, bool MULT, int PG>
double run(int64_t nb, const double* E, const double* mult, int nnode, double* out) {
    const int steps = 32;
    const int64_t waves = nb / steps;
    const int grid = (int)((waves * 64 + 255) / 256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_stream<MODE, MULT, PG><<<grid, 256>>>(nb, steps, E, mult, nnode, out);
    CK(hipEventRecord(a));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) k_stream<MODE, MULT, PG><<<grid, 256>>>(nb, steps, E, mult, nnode, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return (double)nb * 2048.0 * reps / (ms * 1e-3) / 1e9;
}

int main() {
    const int64_t nb = 1555200;  // ~3.2 GB of blocks, the clustered M2L's reads at 1M points
    const int nnode = 87380;
    double *E, *mult, *out;
    CK(hipMalloc(&E, nb * 2048));
    CK(hipMalloc(&mult, (size_t)nnode * 16 * 5 * 8));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(E, 0, nb * 2048));
    CK(hipMemset(mult, 0, (size_t)nnode * 640));
    std::printf("{\"frag\": %.0f, \"line\": %.0f, \"tr\": %.0f, \"frag_pg4\": %.0f, \"line_pg4\": %.0f, ",
                run<0, false, 2>(nb, E, mult, nnode, out), run<1, false, 2>(nb, E, mult, nnode, out),
                run<2, false, 2>(nb, E, mult, nnode, out), run<0, false, 4>(nb, E, mult, nnode, out),
                run<1, false, 4>(nb, E, mult, nnode, out));
    std::printf("\"fragm\": %.0f, \"linem\": %.0f, \"trm\": %.0f, \"unit\": \"GB/s of E blocks\"}\n",
                run<0, true, 2>(nb, E, mult, nnode, out), run<1, true, 2>(nb, E, mult, nnode, out),
                run<2, true, 2>(nb, E, mult, nnode, out));
    std::printf("{\"ms_per_launch\": {\"pg2\": %.3f, \"pg2_pf\": %.3f, \"pg1\": %.3f, \"pg1_pf\": %.3f, \"pg2_w2\": %.3f, \"pg2_pf_w2\": %.3f, \"pg4_w2\": %.3f, \"pg1_pf_w4\": %.3f, \"pg2_w4\": %.3f}}\n",
                run_c<2, false, 3>(nb, E, mult, nnode, out), run_c<2, true, 3>(nb, E, mult, nnode, out),
                run_c<1, false, 3>(nb, E, mult, nnode, out), run_c<1, true, 3>(nb, E, mult, nnode, out),
                run_c<2, false, 2>(nb, E, mult, nnode, out), run_c<2, true, 2>(nb, E, mult, nnode, out),
                run_c<4, false, 2>(nb, E, mult, nnode, out), run_c<1, true, 4>(nb, E, mult, nnode, out),
                run_c<2, false, 4>(nb, E, mult, nnode, out));
    return 0;
}
