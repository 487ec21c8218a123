// solver.hip -- the callers of the hot path: main.cpp's
// forwardOperator u - K_0(sigma_s .* u) (main.cpp:125-136) and the restarted
// GMRES(m) that drives it (gmres.cpp:53-169), with every vector resident in HBM.
// BLAS-1 reductions use a fixed two-level tree so results are deterministic.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "aniso_op.hpp"
#include "arnoldi.hpp"
#include "arnoldi16.hpp"
#include "device_common.hpp"
#include "kernels.hpp"

namespace aniso {

[[noreturn]] void throw_hip(hipError_t e, const char* file, int line);
#define HIP_CHECK(x)                                               \
    do {                                                           \
        hipError_t e__ = (x);                                      \
        if (e__ != hipSuccess) throw_hip(e__, __FILE__, __LINE__); \
    } while (0)

constexpr int kRedBlocks = 512;

// y = alpha x + beta y
__global__ void k_axpby(int64_t n, double alpha, const double* __restrict__ x, double beta, double* __restrict__ y) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = alpha * x[i] + beta * y[i];
}

// z = x - y
__global__ void k_sub(int64_t n, const double* __restrict__ x, const double* __restrict__ y, double* __restrict__ z) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) z[i] = x[i] - y[i];
}

__global__ void __launch_bounds__(256) k_dot_partial(int64_t n, const double* __restrict__ x,
                                                     const double* __restrict__ y, double* __restrict__ part) {
    __shared__ double s[256];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += x[i] * y[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

__global__ void __launch_bounds__(256) k_dot_final(int nb, const double* __restrict__ part, double* __restrict__ out) {
    __shared__ double s[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) acc += part[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = s[0];
}

static unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

// ---- Krylov kernels of the block solve (aniso.m:159-173): classical Gram-Schmidt
// with one reorthogonalisation (CGS2) on device-resident bases.  Every reduction
// has a fixed order (per-block partials, then one block per output), so a solve is
// bitwise reproducible; no host round trip sits inside a step except reading the
// Hessenberg column for the Givens rotations.
constexpr int kDotGroup = 8;  // basis vectors reduced together per pass over w

// part[k * gridDim.x + blk] = sum over this block's chunk of V[k][j] w[j], k < nv
__global__ void __launch_bounds__(256) k_mdot_partial(int64_t n, int nv, const double* __restrict__ V, int64_t ldv,
                                                      const double* __restrict__ w, double* __restrict__ part) {
    __shared__ double red[kDotGroup][256];
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t j0 = (int64_t)blockIdx.x * chunk, j1 = min(n, j0 + chunk);
    for (int k0 = 0; k0 < nv; k0 += kDotGroup) {
        double acc[kDotGroup];
#pragma unroll
        for (int g = 0; g < kDotGroup; ++g) acc[g] = 0.0;
        for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
            const double wj = w[j];
#pragma unroll
            for (int g = 0; g < kDotGroup; ++g)
                if (k0 + g < nv) acc[g] = __builtin_fma(V[(size_t)(k0 + g) * ldv + j], wj, acc[g]);
        }
#pragma unroll
        for (int g = 0; g < kDotGroup; ++g) red[g][threadIdx.x] = acc[g];
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o)
#pragma unroll
                for (int g = 0; g < kDotGroup; ++g) red[g][threadIdx.x] += red[g][threadIdx.x + o];
            __syncthreads();
        }
        if ((int)threadIdx.x < kDotGroup && k0 + (int)threadIdx.x < nv)
            part[(size_t)(k0 + threadIdx.x) * gridDim.x + blockIdx.x] = red[threadIdx.x][0];
        __syncthreads();
    }
}

// out[k] (+)= sum_b part[k * nb + b]: one block per k, a fixed order
__global__ void __launch_bounds__(256) k_mdot_final(int nb, const double* __restrict__ part, int accumulate,
                                                    double* __restrict__ out) {
    __shared__ double r[256];
    const int k = blockIdx.x;
    double a = 0.0;
    for (int b = threadIdx.x; b < nb; b += 256) a += part[(size_t)k * nb + b];
    r[threadIdx.x] = a;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[k] = accumulate ? out[k] + r[0] : r[0];
}

// w[j] += sign * sum_{k < nv} c[k] V[k][j]
__global__ void __launch_bounds__(256) k_maxpy(int64_t n, int nv, const double* __restrict__ V, int64_t ldv,
                                               const double* __restrict__ c, double sign, double* __restrict__ w) {
    extern __shared__ double cs[];
    for (int k = threadIdx.x; k < nv; k += 256) cs[k] = sign * c[k];
    __syncthreads();
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    double a = w[j];
    for (int k = 0; k < nv; ++k) a = __builtin_fma(cs[k], V[(size_t)k * ldv + j], a);
    w[j] = a;
}

// y = a x
__global__ void k_scale(int64_t n, double a, const double* __restrict__ x, double* __restrict__ y) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) y[j] = a * x[j];
}

// y = x / sqrt(*nrm2) (a norm computed on the device; 0 stays 0)
__global__ void k_scale_rsqrt(int64_t n, const double* __restrict__ x, const double* __restrict__ nrm2,
                              double* __restrict__ y) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double s = *nrm2 > 0.0 ? 1.0 / sqrt(*nrm2) : 0.0;
    if (j < n) y[j] = x[j] * s;
}

// orig[perm[k]] = tree[k] (the inverse of launch_permute)
__global__ void k_unpermute(int64_t n, const int* __restrict__ perm, const double* __restrict__ tree,
                            double* __restrict__ orig) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) orig[perm[k]] = tree[k];
}

// ---- the CGS2 sweeps with the basis held in registers (nv <= 48 vectors): one read of
// V per sweep.  Each thread owns elements j of its block's chunk;
// the per-block sums of the NV products reduce by xor shuffles inside a wave and then
// over the 4 waves in a fixed order (deterministic).
template <int NV>
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// per-block sums of acc[k] (k < nv) into part[k * gridDim.x + blockIdx.x], and with SQ
// of acc[NA - 1] into row nv: wave sums by xor shuffles, then the 4 waves in a fixed order
template <int NA, bool SQ>
__device__ __forceinline__ void block_partials(const double (&acc)[NA], int nv, double* red, double* part) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int ND = SQ ? NA - 1 : NA;
#pragma unroll
    for (int k = 0; k < ND; ++k)
        if (k < nv) {
            const double v = wave_sum<0>(acc[k]);
            if (lane == 0) red[wv * NA + k] = v;
        }
    if constexpr (SQ) {
        const double v = wave_sum<0>(acc[NA - 1]);
        if (lane == 0) red[wv * NA + NA - 1] = v;
    }
    __syncthreads();
    const int rows = SQ ? nv + 1 : nv;
    for (int k = threadIdx.x; k < rows; k += blockDim.x) {
        const int i = SQ && k == nv ? NA - 1 : k;
        part[(size_t)k * gridDim.x + blockIdx.x] = ((red[i] + red[NA + i]) + red[2 * NA + i]) + red[3 * NA + i];
    }
}

// pass 1: part[k][blk] = sum over the block's chunk of V[k][j] w[j]
template <int NV>
__global__ void __launch_bounds__(256) k_cgs_dot(int64_t n, int nv, const double* __restrict__ V, int64_t ldv,
                                                 const double* __restrict__ w, double* __restrict__ part) {
    __shared__ double red[4 * NV];
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t j0 = (int64_t)blockIdx.x * chunk, j1 = min(n, j0 + chunk);
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
        double v[NV];  // every load of the element in flight before the products
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = k < nv ? V[(size_t)k * ldv + j] : 0.0;
        const double wj = w[j];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < nv) acc[k] = __builtin_fma(v[k], wj, acc[k]);
    }
    block_partials<NV, false>(acc, nv, red, part);
}

// pass 2 / 3: w[j] -= sum_k c[k] V[k][j] (k_maxpy's order), then the products of the
// updated w with the same V[k][j] (DOT: the reorthogonalisation's h = V^T w, rows
// 0 .. nv-1) and its square (||w||^2: row nv with DOT, row 0 without)
template <int NV, bool DOT>
__global__ void __launch_bounds__(256) k_cgs_update(int64_t n, int nv, const double* __restrict__ V, int64_t ldv,
                                                    const double* __restrict__ c, double* __restrict__ w,
                                                    double* __restrict__ part) {
    constexpr int NA = DOT ? NV + 1 : 1;
    __shared__ double red[4 * NA];
    __shared__ double cs[NV];
    for (int k = threadIdx.x; k < nv; k += blockDim.x) cs[k] = -c[k];
    __syncthreads();
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t j0 = (int64_t)blockIdx.x * chunk, j1 = min(n, j0 + chunk);
    double acc[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) acc[k] = 0.0;
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
        double v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = k < nv ? V[(size_t)k * ldv + j] : 0.0;
        double a = w[j];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < nv) a = __builtin_fma(cs[k], v[k], a);
        w[j] = a;
        if constexpr (DOT) {
#pragma unroll
            for (int k = 0; k < NV; ++k)
                if (k < nv) acc[k] = __builtin_fma(v[k], a, acc[k]);
        }
        acc[NA - 1] = __builtin_fma(a, a, acc[NA - 1]);
    }
    if constexpr (DOT) block_partials<NA, true>(acc, nv, red, part);
    else block_partials<1, false>(acc, 1, red, part);
}

constexpr int kCgsMaxRegs = 48;  // basis vectors the register-held sweeps take

constexpr int kMdotBlocks = 2048;  // partial sums per reduction (per-block chunks of ~2.5K elements at 1M x 5)

struct Krylov {
    int64_t n;
    hipStream_t s;
    double* part;  // kMdotBlocks x (restart + 1)
    // out[0 .. nv) (+)= V[0 .. nv)^T w
    void mdot(int nv, const double* V, int64_t ldv, const double* w, double* out, bool accumulate) {
        k_mdot_partial<<<kMdotBlocks, 256, 0, s>>>(n, nv, V, ldv, w, part);
        k_mdot_final<<<nv, 256, 0, s>>>(kMdotBlocks, part, accumulate ? 1 : 0, out);
    }
    void maxpy(int nv, const double* V, int64_t ldv, const double* c, double sign, double* w) {
        k_maxpy<<<nblk(n), 256, (size_t)nv * sizeof(double), s>>>(n, nv, V, ldv, c, sign, w);
    }
    // the three sweeps of a CGS2 step over nv basis vectors: h = V^T w; w -= V h with
    // h2 = V^T w from the same read of V; w -= V h2 with ||w||^2 (one read of V each
    // for nv <= kCgsMaxRegs, else the two-pass kernels above)
    template <typename F>
    static void nv_dispatch(int nv, F&& f) {
        if (nv <= 8) f(std::integral_constant<int, 8>{});
        else if (nv <= 16) f(std::integral_constant<int, 16>{});
        else if (nv <= 32) f(std::integral_constant<int, 32>{});
        else f(std::integral_constant<int, kCgsMaxRegs>{});
    }
    void dot(int nv, const double* V, int64_t ldv, const double* w, double* out) {
        if (nv > kCgsMaxRegs) return mdot(nv, V, ldv, w, out, false);
        nv_dispatch(nv, [&](auto c) {
            k_cgs_dot<decltype(c)::value><<<kMdotBlocks, 256, 0, s>>>(n, nv, V, ldv, w, part);
        });
        k_mdot_final<<<nv, 256, 0, s>>>(kMdotBlocks, part, 0, out);
    }
    // w -= V c, then out[k] = V_k . w (k < nv) and out[nv] = w . w
    void updateDot(int nv, const double* V, int64_t ldv, const double* c, double* w, double* out) {
        if (nv > kCgsMaxRegs) {
            maxpy(nv, V, ldv, c, -1.0, w);
            mdot(nv, V, ldv, w, out, false);
            return mdot(1, w, ldv, w, out + nv, false);
        }
        nv_dispatch(nv, [&](auto cc) {
            k_cgs_update<decltype(cc)::value, true><<<kMdotBlocks, 256, 0, s>>>(n, nv, V, ldv, c, w, part);
        });
        k_mdot_final<<<nv + 1, 256, 0, s>>>(kMdotBlocks, part, 0, out);
    }
    void updateNorm(int nv, const double* V, int64_t ldv, const double* c, double* w, double* nrm2) {
        if (nv > kCgsMaxRegs) {
            maxpy(nv, V, ldv, c, -1.0, w);
            return mdot(1, w, ldv, w, nrm2, false);
        }
        nv_dispatch(nv, [&](auto cc) {
            k_cgs_update<decltype(cc)::value, false><<<kMdotBlocks, 256, 0, s>>>(n, nv, V, ldv, c, w, part);
        });
        k_mdot_final<<<1, 256, 0, s>>>(kMdotBlocks, part, 0, nrm2);
    }
};

struct DeviceBlas {
    int64_t n;
    hipStream_t s;
    double* part;
    double* res;
    double dot(const double* x, const double* y) {
        k_dot_partial<<<kRedBlocks, 256, 0, s>>>(n, x, y, part);
        k_dot_final<<<1, 256, 0, s>>>(kRedBlocks, part, res);
        double h = 0;
        HIP_CHECK(hipMemcpyAsync(&h, res, sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        return h;
    }
    double nrm2(const double* x) { return std::sqrt(dot(x, x)); }
    void axpby(double a, const double* x, double b, double* y) { k_axpby<<<nblk(n), 256, 0, s>>>(n, a, x, b, y); }
};

// forwardOperator (main.cpp:125-136): out = u - K_0(sigma_s .* u)
void Operator::forwardDev(const double* u, double* out, hipStream_t s) {
    if (plan.nranks != 1) throw std::logic_error("forward operator on a sharded handle: gather first");
    ensureDevice();
    apply(u, false, dSigmaT.as<double>(), 0, dTmp2.as<double>(), false, s, kStageAll);  // sigma_s .* u inside the up pass
    k_sub<<<nblk(geo.N), 256, 0, s>>>(geo.N, u, dTmp2.as<double>(), out);
}

// main.cpp:121-141: rhs = K_0 q; GMRES(forwardOperator, x, rhs, m, maxit, tol).
// Mirrors gmres.cpp:53-169 (MGS, Givens, restart with Update).  Returns the
// iteration count j on convergence and -j otherwise; hist gets the residual
// printed at the start of every inner iteration plus the final one.
int Operator::gmresHost(const double* q, double* xh, int m, int maxit, double tol, double* hist, int maxhist,
                        double* finalResid) {
    if (m < 1 || maxit < 0) throw std::invalid_argument("GMRES needs m >= 1 and maxit >= 0");
    if (!modeCached(0)) throw std::runtime_error("GMRES before cache(0)");
    ensureDevice();
    const int64_t N = geo.N;
    hipStream_t s = own;
    DevBuf bq, bb, br, bp, bx, bpart, bres;
    bq.upload(q, N * sizeof(double));
    bx.upload(xh, N * sizeof(double));
    bb.alloc(N * sizeof(double));
    br.alloc(N * sizeof(double));
    bp.alloc(N * sizeof(double));
    bpart.alloc(kRedBlocks * sizeof(double));
    bres.alloc(sizeof(double));
    std::vector<DevBuf> v(m + 1);
    for (auto& vi : v) vi.alloc(N * sizeof(double));
    DeviceBlas B{N, s, bpart.as<double>(), bres.as<double>()};
    double* b = bb.as<double>();
    double* r = br.as<double>();
    double* p = bp.as<double>();
    double* x = bx.as<double>();
    mappingDev(bq.as<double>(), 0, b, s, kStageAll);  // rhs = apply_mapping(charge)
    const int ld = m + 1;
    std::vector<double> H((size_t)ld * ld, 0.0), sv(ld, 0.0), cs(ld, 0.0), sn(ld, 0.0);
    int nh = 0, ret;
    auto rot = [](double& dx, double& dy, double c, double sn_) {
        double t = c * dx + sn_ * dy;
        dy = -sn_ * dx + c * dy;
        dx = t;
    };
    auto gen = [](double dx, double dy, double& c, double& sn_) {
        if (dy == 0.0) { c = 1.0; sn_ = 0.0; }
        else if (std::fabs(dy) > std::fabs(dx)) { double t = dx / dy; sn_ = 1.0 / std::sqrt(1.0 + t * t); c = t * sn_; }
        else { double t = dy / dx; c = 1.0 / std::sqrt(1.0 + t * t); sn_ = t * c; }
    };
    auto update = [&](int k) {  // Update (gmres.cpp:12-24)
        std::vector<double> y(sv.begin(), sv.begin() + k + 1);
        for (int i = k; i >= 0; i--) {
            y[i] /= H[i + (size_t)i * ld];
            for (int j2 = i - 1; j2 >= 0; j2--) y[j2] -= H[j2 + (size_t)i * ld] * y[i];
        }
        for (int j2 = 0; j2 <= k; j2++) B.axpby(y[j2], v[j2].as<double>(), 1.0, x);
    };
    double normb = B.nrm2(b);
    forwardDev(x, p, s);
    k_sub<<<nblk(N), 256, 0, s>>>(N, b, p, r);
    double beta = B.nrm2(r), resid;
    if (normb == 0.0) normb = 1;
    int i = 0, j = 1;
    if ((resid = beta / normb) <= tol) {
        ret = 0;
        goto done;
    }
    while (j <= maxit) {
        HIP_CHECK(hipMemcpyAsync(v[0].p, r, N * sizeof(double), hipMemcpyDeviceToDevice, s));
        B.axpby(0.0, r, 1.0 / beta, v[0].as<double>());
        std::fill(sv.begin(), sv.end(), 0.0);
        sv[0] = beta;
        for (i = 0; i < m && j <= maxit; i++, j++) {
            if (hist && nh < maxhist) hist[nh++] = resid;
            forwardDev(v[i].as<double>(), p, s);
            for (int k = 0; k <= i; k++) {
                double h = B.dot(p, v[k].as<double>());
                H[k + (size_t)i * ld] = h;
                B.axpby(-h, v[k].as<double>(), 1.0, p);
            }
            double hn = B.nrm2(p);
            H[(i + 1) + (size_t)i * ld] = hn;
            HIP_CHECK(hipMemcpyAsync(v[i + 1].p, p, N * sizeof(double), hipMemcpyDeviceToDevice, s));
            B.axpby(0.0, p, 1.0 / hn, v[i + 1].as<double>());
            for (int k = 0; k < i; k++) rot(H[k + (size_t)i * ld], H[(k + 1) + (size_t)i * ld], cs[k], sn[k]);
            gen(H[i + (size_t)i * ld], H[(i + 1) + (size_t)i * ld], cs[i], sn[i]);
            rot(H[i + (size_t)i * ld], H[(i + 1) + (size_t)i * ld], cs[i], sn[i]);
            rot(sv[i], sv[i + 1], cs[i], sn[i]);
            if ((resid = std::fabs(sv[i + 1]) / normb) < tol) {
                update(i);
                ret = j;
                goto done;
            }
        }
        update(i - 1);
        forwardDev(x, p, s);
        k_sub<<<nblk(N), 256, 0, s>>>(N, b, p, r);
        beta = B.nrm2(r);
        if ((resid = beta / normb) < tol) {
            ret = j;
            goto done;
        }
    }
    ret = -j;
done:
    if (hist && nh < maxhist) hist[nh++] = resid;
    if (finalResid) *finalResid = resid;
    HIP_CHECK(hipMemcpyAsync(xh, x, N * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    checkDeviceErrors();
    return ret;
}

// aniso.m:159-173: u = gmres(A, rhs, restart, tol, maxit) with A(x) = x - mforward(x)
// (aniso.m:155) on the nb = ks stacked blocks.  MATLAB's restarted GMRES semantics:
// x0 = the given guess, at most maxit cycles of at most `restart` steps, converged
// when ||rhs - A x|| / ||rhs|| <= tol (the estimate inside a cycle, confirmed by the
// explicit residual at its end).  The vectors are permuted once into tree order and
// every Krylov vector ((restart + 1) x ks x N doubles) stays in HBM; orthogonalisation
// is CGS2 on the device.  rhs / x: device, original order, block b at b * N.
// Returns the total step count (negative if not converged); hist gets the relative
// residual estimate after every step.
// The CGS2 sweeps as library primitives for a caller's own Krylov loop (the sharded
// GMRES of aniso_amd.solve.gmres_dist reduces their outputs over the ranks between
// the calls): out[k] = V_k . w; and w -= V c followed by out[k] = V_k . w, out[nv] =
// w . w (dots) or out[0] = w . w.  Device pointers, on stream s.
void Operator::krylovDot(int64_t n, int nv, const double* V, int64_t ldv, const double* w, double* out,
                         hipStream_t s) {
    if (n < 0 || nv < 1 || ldv < n) throw std::invalid_argument("krylov dot: bad sizes");
    ensureDevice();
    dKryPart.alloc(std::max(dKryPart.bytes, (size_t)kMdotBlocks * (nv + 2) * sizeof(double)));
    Krylov kr{n, s, dKryPart.as<double>()};
    kr.dot(nv, V, ldv, w, out);
}

void Operator::krylovUpdate(int64_t n, int nv, const double* V, int64_t ldv, const double* c, double* w,
                            double* out, bool dots, hipStream_t s) {
    if (n < 0 || nv < 1 || ldv < n) throw std::invalid_argument("krylov update: bad sizes");
    ensureDevice();
    dKryPart.alloc(std::max(dKryPart.bytes, (size_t)kMdotBlocks * (nv + 2) * sizeof(double)));
    Krylov kr{n, s, dKryPart.as<double>()};
    if (dots) kr.updateDot(nv, V, ldv, c, w, out);
    else kr.updateNorm(nv, V, ldv, c, w, out);
}

// ---- DCGS2 Arnoldi on a never-rewritten basis (arnoldi.hpp): the library primitives
// (aniso_arnoldi_*) and the block solve on them.  dKryPart holds the sweeps' partial
// sums (arn::kParts per row).
int64_t arn_state_doubles(int m) { return arn::Layout(m).total; }

static void check_arnoldi(int m, int j) {
    if (m < 1 || j < 0 || j >= m) throw std::invalid_argument("arnoldi: need 0 <= j < m");
}

// the small kernels' fast paths stage up to ~100 KB of LDS: their dynamic limit is
// raised once per device (a function attribute binds to the device current at the
// call), checked, before any launch of them on that device
static void arn_small_kernel_attrs() {
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return;
    for (const void* f : {(const void*)arn::k_arn_coef, (const void*)arn::k_arn_column}) {
        e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 136 * 1024);
        if (e != hipSuccess) throw_hip(e, __FILE__, __LINE__);
    }
    done.fetch_or(bit, std::memory_order_acq_rel);
}

// dKryPart for sweeps of `rows` rows.  DevBuf::alloc frees and reallocates (a device
// synchronisation) on every size change, so it grows geometrically; the Arnoldi entry
// points that know the restart length size it for the whole cycle at once
void Operator::arnoldiParts(int rows) {
    arn_small_kernel_attrs();
    const size_t need = (size_t)arn::kParts * (rows + 2) * sizeof(double);
    if (need > dKryPart.bytes) dKryPart.alloc(std::max(need, 2 * dKryPart.bytes));
}

void Operator::arnoldiBegin(int64_t n, int m, const double* V, int64_t ldv, double* st, const double* rr,
                            double normb, double* status, hipStream_t s) {
    if (m < 1 || n < 0 || ldv < n || !(normb > 0.0)) throw std::invalid_argument("arnoldi begin: bad sizes or |b|");
    ensureDevice();
    if (rr) {
        arn::k_arn_begin<<<1, arn::kThreads, 0, s>>>(m, st, rr, 1, normb, status);
        HIP_LAUNCH_CHECK();
        return;
    }
    arnoldiParts(m + 2);
    arn::launch_project(n, 1, V, ldv, V, dKryPart.as<double>(), s);
    arn::k_arn_begin<<<1, arn::kThreads, 0, s>>>(m, st, dKryPart.as<double>(), arn::kParts, normb, status);
    HIP_LAUNCH_CHECK();
}

void Operator::arnoldiStep(int64_t n, int m, int j, double* V, int64_t ldv, const double* w, double* st,
                           double* status, hipStream_t s) {
    check_arnoldi(m, j);
    if (n < 0 || ldv < n) throw std::invalid_argument("arnoldi step: bad sizes");
    ensureDevice();
    arnoldiParts(m + 2);
    double* part = dKryPart.as<double>();
    arn::launch_project(n, j + 1, V, ldv, w, part, s);
    arn::k_arn_coef<<<1, arn::kThreads, arn::coef_lds(j), s>>>(m, j, st, part, arn::kParts);
    HIP_LAUNCH_CHECK();
    arn::launch_update(n, j + 1, V, ldv, w, st, m, part, s);
    arn::k_arn_column<<<1, arn::kThreads, arn::column_lds(j), s>>>(m, j, st, part, arn::kParts, status);
    HIP_LAUNCH_CHECK();
}

void Operator::arnoldiProject(int64_t n, int j, const double* V, int64_t ldv, const double* w, double* out,
                              hipStream_t s) {
    if (n < 0 || j < 0 || ldv < n) throw std::invalid_argument("arnoldi project: bad sizes");
    ensureDevice();
    arnoldiParts(j + 1);
    arn::launch_project(n, j + 1, V, ldv, w, dKryPart.as<double>(), s);
    arn::k_arn_rows<<<1, arn::kThreads, (size_t)(j + 1) * sizeof(double), s>>>(dKryPart.as<double>(), arn::kParts,
                                                                                 j + 1, out);
    HIP_LAUNCH_CHECK();
}

void Operator::arnoldiCoef(int m, int j, double* st, const double* red, hipStream_t s) {
    check_arnoldi(m, j);
    ensureDevice();
    arn_small_kernel_attrs();
    arn::k_arn_coef<<<1, arn::kThreads, arn::coef_lds(j), s>>>(m, j, st, red, 1);
    HIP_LAUNCH_CHECK();
}

void Operator::arnoldiUpdate(int64_t n, int m, int j, double* V, int64_t ldv, const double* w, const double* st,
                             double* out, hipStream_t s) {
    check_arnoldi(m, j);
    if (n < 0 || ldv < n) throw std::invalid_argument("arnoldi update: bad sizes");
    ensureDevice();
    arnoldiParts(m + 2);
    arn::launch_update(n, j + 1, V, ldv, w, st, m, dKryPart.as<double>(), s);
    arn::k_arn_rows<<<1, arn::kThreads, (size_t)(j + 2) * sizeof(double), s>>>(dKryPart.as<double>(), arn::kParts,
                                                                                 j + 2, out);
    HIP_LAUNCH_CHECK();
}

void Operator::arnoldiColumn(int m, int j, double* st, const double* red, double* status, hipStream_t s) {
    check_arnoldi(m, j);
    ensureDevice();
    arn_small_kernel_attrs();
    arn::k_arn_column<<<1, arn::kThreads, arn::column_lds(j), s>>>(m, j, st, red, 1, status);
    HIP_LAUNCH_CHECK();
}

void Operator::arnoldiSolution(int64_t n, int m, int used, const double* V, int64_t ldv, double* st, double* x,
                               hipStream_t s) {
    if (m < 1 || used < 0 || used > m || n < 0 || ldv < n) throw std::invalid_argument("arnoldi solution: bad sizes");
    ensureDevice();
    if (used == 0) return;
    arn::k_arn_solve<<<1, arn::kThreads, arn::solve_lds(used), s>>>(m, used, st);
    HIP_LAUNCH_CHECK();
    if (n > 0)
        arn::k_arn_axpy<<<nblk(n), arn::kThreads, (size_t)used * sizeof(double), s>>>(n, used, V, ldv,
                                                                                        st + arn::Layout(m).y, x);
    HIP_LAUNCH_CHECK();
}

// aniso.m:159-173: u = gmres(A, rhs, restart, tol, maxit) with A(x) = x - mforward(x)
// (aniso.m:155) on the nb = ks stacked blocks.  MATLAB's restarted GMRES semantics:
// x0 = the given guess, at most maxit cycles of at most `restart` steps, converged
// when ||rhs - A x|| / ||rhs|| <= tol (the estimate inside a cycle, confirmed by the
// explicit residual at its end).  The vectors are permuted once into tree order and
// every Krylov vector ((restart + 1) x ks x N doubles) stays in HBM; the Arnoldi
// process is DCGS2 on the device (arnoldi.hpp): per step the matvec, two sweeps over
// the basis and two one-block kernels; the host reads one status word per step
// while the GPU already runs the next step's matvec.  rhs / x: device, original
// order, block b at b * N.  Returns the total step count (negative if not converged);
// hist gets the relative residual estimate after every step.
int Operator::blockSolveDev(const double* rhs, double* x, int restart, double tol, int maxit, double* hist,
                            int maxhist, double* relresOut, hipStream_t s) {
    if (plan.nranks != 1) throw std::logic_error("block solve on a sharded handle");
    if (!coeffSet) throw std::runtime_error("block solve before setCoeff");
    for (int m = 0; m < kernelSize; ++m)
        if (!modes[m].ready) throw std::runtime_error("block solve before cache(" + std::to_string(m) + ")");
    if (restart < 1 || maxit < 1 || !(tol > 0.0)) throw std::invalid_argument("block solve needs restart >= 1, maxit >= 1, tol > 0");
    ensureDevice();
    checkDeviceErrors();
    const int64_t N = geo.N, L = (int64_t)ks * N;
    const int m = restart;
    const arn::Layout lay(m);
    DevBuf bB, bX, bW, bV, bSt;
    bB.alloc(L * sizeof(double));
    bX.alloc(L * sizeof(double));
    bW.alloc(L * sizeof(double));
    bV.alloc((size_t)(m + 1) * L * sizeof(double));
    bSt.alloc((size_t)lay.total * sizeof(double));
    arnoldiParts(m + 2);
    double *b = bB.as<double>(), *xt = bX.as<double>(), *w = bW.as<double>();
    double* V = bV.as<double>();
    double* st = bSt.as<double>();
    const int* perm = dPerm.as<int>();
    for (int k = 0; k < ks; ++k) {  // tree order: the operator needs no permutation gathers
        launch_permute(N, perm, rhs + (size_t)k * N, b + (size_t)k * N, s);
        launch_permute(N, perm, x + (size_t)k * N, xt + (size_t)k * N, s);
    }
    // the status word {relres, r', steps} in mapped host memory: the column kernel
    // stores it there and the host waits for an event behind it, not a stream drain
    struct HostStat {
        double* p = nullptr;
        hipEvent_t ev = nullptr;
        ~HostStat() {
            if (p) (void)hipHostFree(p);
            if (ev) (void)hipEventDestroy(ev);
        }
    } hs;
    HIP_CHECK(hipHostMalloc((void**)&hs.p, 4 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(hipEventCreateWithFlags(&hs.ev, hipEventDisableTiming));
    double* stat = nullptr;
    HIP_CHECK(hipHostGetDevicePointer((void**)&stat, hs.p, 0));
    auto post = [&] { HIP_CHECK(hipEventRecord(hs.ev, s)); };
    auto sumsq = [&](const double* v) {  // |v|^2 on the host (once per solve)
        arn::launch_project(L, 1, v, L, v, dKryPart.as<double>(), s);
        arn::k_arn_rows<<<1, arn::kThreads, sizeof(double), s>>>(dKryPart.as<double>(), arn::kParts, 1, stat);
        post();
        HIP_CHECK(hipEventSynchronize(hs.ev));
        return hs.p[0];
    };
    // a fused-launch time-out (recoverTopTimeout) re-runs the apply it spoiled on the
    // tier launches, and the rest of the solve keeps them
    struct Restore {
        bool& f;
        bool v;
        ~Restore() { f = v; }
    } restore{forceUnfused, forceUnfused}, own{ownTimeline, ownTimeline};
    ownTimeline = true;  // the look-ahead matvec may be enqueued after a spoiled one: recovered below
    const double normb = std::sqrt(sumsq(b));
    // A 0 = 0: a zero initial guess needs no matvec for its residual
    bool xZero = normb > 0.0 && sumsq(xt) == 0.0;
    // r = b - A x into V[0], then the cycle's start; returns |r| / |b|
    auto residual = [&] {
        for (int tries = 0;; ++tries) {
            if (xZero) {
                HIP_CHECK(hipMemcpyAsync(V, b, L * sizeof(double), hipMemcpyDeviceToDevice, s));
            } else {
                blockOpDev(2, xt, N, w, N, true, s);
                k_sub<<<nblk(L), 256, 0, s>>>(L, b, w, V);
            }
            arnoldiBegin(L, m, V, L, st, nullptr, normb, stat, s);
            post();
            HIP_CHECK(hipEventSynchronize(hs.ev));
            if (!recoverTopTimeout(s) || tries > 0) return hs.p[0];
        }
    };
    int nh = 0, total = 0;
    double relres = 0.0;
    bool conv = false;
    if (normb == 0.0) {
        HIP_CHECK(hipMemsetAsync(xt, 0, L * sizeof(double), s));
        conv = true;
    } else {
        relres = residual();
        conv = relres <= tol;
        std::vector<double> hrel;
        for (int cyc = 0; cyc < maxit && !conv; ++cyc) {
            if (hs.p[1] == 0.0) break;  // |r| = 0 in floating point
            int used = 0;
            bool ahead = false;  // the matvec of V[j] is already enqueued
            hrel.clear();
            for (int j = 0; j < m; ++j) {
                double* vj = V + (size_t)j * L;
                if (!ahead) blockOpDev(2, vj, N, w, N, true, s);
                arnoldiStep(L, m, j, V, L, w, st, stat, s);
                post();
                // the next step's matvec goes in before the host reads the status: the GPU
                // runs it while the host decides (wasted once per cycle, at the step that
                // converges) -- except where the residual estimate is predicted to reach tol
                // at this step (geometric extrapolation of the last two estimates, 10x margin)
                bool near = false;
                if (hrel.size() >= 2) {
                    const double q = std::min(1.0, hrel.back() / hrel[hrel.size() - 2]);
                    near = hrel.back() * q <= 10.0 * tol;
                } else if (!hrel.empty()) {
                    near = hrel.back() <= 10.0 * tol;
                }
                ahead = j + 1 < m && !near;
                if (ahead) blockOpDev(2, V + (size_t)(j + 1) * L, N, w, N, true, s);
                HIP_CHECK(hipEventSynchronize(hs.ev));
                if (recoverTopTimeout(s)) {
                    // this step's matvec (or the look-ahead one) ran on an invalid fused launch:
                    // the cycle ends before this step (columns 0 .. j - 1 are valid) and restarts
                    // from its update on the tier launches
                    ahead = false;
                    break;
                }
                const double rel = hs.p[0], rnext = hs.p[1];
                if (hs.p[2] != (double)(j + 1))  // the column kernel of this step did not run
                    throw std::runtime_error("block solve: Arnoldi step " + std::to_string(j) + " left no status");
                ++total;
                used = j + 1;
                relres = rel;
                hrel.push_back(rel);
                if (hist && nh < maxhist) hist[nh++] = rel;
                if (rel <= tol || rnext == 0.0) break;  // converged (estimate) or lucky breakdown
            }
            arnoldiSolution(L, m, used, V, L, st, xt, s);  // x += P T R^-1 g
            xZero = xZero && used == 0;
            relres = residual();
            conv = relres <= tol;
        }
    }
    for (int k = 0; k < ks; ++k)
        k_unpermute<<<nblk(N), 256, 0, s>>>(N, perm, xt + (size_t)k * N, x + (size_t)k * N);
    HIP_CHECK(hipStreamSynchronize(s));
    ownTimeline = false;
    checkDeviceErrors();  // every apply was checked at its recovery point: a flag here is new
    if (relresOut) *relresOut = relres;
    return conv ? total : -std::max(total, 1);
}

// Config 5 (main.cpp:121-141 for 16 right-hand sides): A X = B with
// A(u) = u - K_0(sigma_s .* u), fp64 iterative refinement over fp32 inner GMRES(m)
// solves -- the algorithm of aniso_amd.solve.gmres_mixed, every step in the library:
//   outer: R = B - A64 X (the fp64 16-RHS MFMA operator), rel_c = |R_c| / |B_c|; stop
//          when every rel_c <= tol (or after maxOuter refinements); X += inner(R);
//   inner: GMRES(m) per column on an fp32 basis (arnoldi16.hpp: the DCGS2 Arnoldi of
//          the block solve, 16 columns in lockstep), the fp32 16-RHS MFMA operator,
//          to |g_c| <= innerTol |R_c| for every column, at most maxCycles cycles.
// B, X: 16 rows of N doubles (original order, strides ldb / ldx; X is written, the
// initial guess is 0); device pointers, stream s.  Returns the inner steps; *outer the
// refinements; rel: the 16 final relative residuals.
int Operator::solve16Mixed(const double* B, int64_t ldb, double* X, int64_t ldx, int m, double tol, double innerTol,
                           int maxOuter, int maxCycles, int* outerOut, double* rel, hipStream_t s) {
    using namespace arn16;
    if (plan.nranks != 1) throw std::logic_error("16-RHS solve on a sharded handle");
    if (!coeffSet) throw std::runtime_error("16-RHS solve before setCoeff");
    if (!modes[0].ready) throw std::runtime_error("16-RHS solve before cache(0)");
    if (m < 1 || m >= kMaxRows) throw std::invalid_argument("16-RHS solve: restart must be in [1, 47]");
    if (!(tol > 0.0) || !(innerTol > 0.0) || maxOuter < 0 || maxCycles < 1)
        throw std::invalid_argument("16-RHS solve needs tol, inner_tol > 0, max_outer >= 0, max_cycles >= 1");
    const int64_t N = geo.N, n16 = KC * N;
    if (ldb < N || ldx < N) throw std::invalid_argument("16-RHS solve: leading dimension below N");
    ensureDevice();
    checkDeviceErrors();
    const arn::Layout lay(m);
    const int64_t sts = lay.total;
    arn::ColArgs ca = kCols;
    ca.sts = sts;
    auto grow = [](DevBuf& b, size_t bytes) {
        if (b.bytes < bytes) b.alloc(bytes);
    };
    grow(s16B, n16 * sizeof(double));
    grow(s16X, n16 * sizeof(double));
    grow(s16R, n16 * sizeof(double));
    grow(s16W, n16 * sizeof(double));
    grow(s16D, n16 * sizeof(double));
    grow(s16Df, n16 * sizeof(float));
    grow(s16W32, n16 * sizeof(float));
    grow(s16V, (size_t)(m + 1) * n16 * sizeof(float));
    grow(s16St, (size_t)KC * sts * sizeof(double));
    grow(s16Part, (size_t)kParts * KC * (m + 2) * sizeof(double));
    grow(s16R0, KC * sizeof(double));
    arn_small_kernel_attrs();
    double *Bt = s16B.as<double>(), *Xt = s16X.as<double>(), *R = s16R.as<double>(), *W = s16W.as<double>();
    double *D = s16D.as<double>(), *st = s16St.as<double>(), *part = s16Part.as<double>(), *r0d = s16R0.as<double>();
    float *Df = s16Df.as<float>(), *W32 = s16W32.as<float>(), *V = s16V.as<float>();
    const int* perm = dPerm.as<int>();
    // status words in mapped host memory: per column {relres, r', steps, -}, then 16 sums
    struct HostStat {
        double* p = nullptr;
        hipEvent_t ev = nullptr;
        ~HostStat() {
            if (p) (void)hipHostFree(p);
            if (ev) (void)hipEventDestroy(ev);
        }
    } hs;
    HIP_CHECK(hipHostMalloc((void**)&hs.p, 5 * KC * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(hipEventCreateWithFlags(&hs.ev, hipEventDisableTiming));
    double* stat = nullptr;
    HIP_CHECK(hipHostGetDevicePointer((void**)&stat, hs.p, 0));
    double* sums = stat + 4 * KC;
    const double* hsums = hs.p + 4 * KC;
    auto wait = [&] {
        HIP_CHECK(hipEventRecord(hs.ev, s));
        HIP_CHECK(hipEventSynchronize(hs.ev));
    };
    auto colsums = [&] {  // the one-row partials in `part` -> hsums[c]
        k16_rows<<<KC, arn::kThreads, 0, s>>>(part, sums);
        HIP_LAUNCH_CHECK();
        wait();
    };
    const unsigned g16 = nblk(n16);
    k16_gather<<<g16, 256, 0, s>>>(N, perm, B, ldb, Bt);
    k16_sub_norm<double><<<kParts, kT, 0, s>>>(n16, Bt, nullptr, R, nullptr, part);  // R = B (X = 0)
    HIP_LAUNCH_CHECK();
    HIP_CHECK(hipMemsetAsync(Xt, 0, n16 * sizeof(double), s));
    colsums();
    double bn[KC], rn[KC], r0[KC];
    for (int c = 0; c < KC; ++c) bn[c] = std::sqrt(hsums[c]);
    int outer = 0, inner = 0;
    for (;; ++outer) {
        if (outer > 0) {
            mrhs64Dev(0, true, Xt, W, s);  // W = X - K_0(sigma_s .* X), fp64
            k16_sub_norm<double><<<kParts, kT, 0, s>>>(n16, Bt, W, R, nullptr, part);
            HIP_LAUNCH_CHECK();
            colsums();
        }
        bool all = true;
        for (int c = 0; c < KC; ++c) {
            rn[c] = std::sqrt(hsums[c]);
            rel[c] = bn[c] > 0.0 ? rn[c] / bn[c] : 0.0;
            all = all && rel[c] <= tol;
        }
        if (all || outer == maxOuter) break;
        for (int c = 0; c < KC; ++c) r0[c] = rn[c] > 0.0 ? rn[c] : 1.0;
        HIP_CHECK(hipMemcpyAsync(r0d, r0, KC * sizeof(double), hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemsetAsync(D, 0, n16 * sizeof(double), s));
        int its = 0;
        for (int cyc = 0; cyc < maxCycles; ++cyc) {
            // the cycle's residual R - A32 D into V[0] (fp32) and its norm per column
            if (its > 0) {
                k16_round<<<g16, 256, 0, s>>>(n16, D, Df);
                forwardF32Dev(Df, W32, s);
                k16_sub_norm<float><<<kParts, kT, 0, s>>>(n16, R, W32, nullptr, V, part);
            } else {
                k16_sub_norm<double><<<kParts, kT, 0, s>>>(n16, R, nullptr, nullptr, V, part);
            }
            HIP_LAUNCH_CHECK();
            arn::k_arn_begin<<<KC, arn::kThreads, 0, s>>>(m, st, part, kParts, 1.0, stat, ca, r0d);
            HIP_LAUNCH_CHECK();
            wait();
            bool done = true;
            for (int c = 0; c < KC; ++c) done = done && hs.p[4 * c] <= innerTol;
            if (done) break;
            int used = 0;
            bool ahead = false;
            std::vector<double> hrel;
            for (int j = 0; j < m; ++j) {
                float* vj = V + (size_t)j * n16;
                if (!ahead) forwardF32Dev(vj, W32, s);
                rows_dispatch(j + 1, [&](auto c) {
                    k16_project<decltype(c)::value><<<kParts, kT, 0, s>>>(n16, j + 1, V, n16, W32, part);
                });
                HIP_LAUNCH_CHECK();
                arn::k_arn_coef<<<KC, arn::kThreads, arn::coef_lds(j), s>>>(m, j, st, part, kParts, ca);
                HIP_LAUNCH_CHECK();
                rows_dispatch(j + 1, [&](auto c) {
                    k16_update<decltype(c)::value><<<kParts, kT, 0, s>>>(n16, j + 1, V, n16, W32, st, sts, m, part);
                });
                HIP_LAUNCH_CHECK();
                arn::k_arn_column<<<KC, arn::kThreads, arn::column_lds(j), s>>>(m, j, st, part, kParts, stat, ca);
                HIP_LAUNCH_CHECK();
                HIP_CHECK(hipEventRecord(hs.ev, s));
                // the next step's matvec before the host reads the estimates (as blockSolveDev)
                bool near = false;
                if (hrel.size() >= 2) near = hrel.back() * std::min(1.0, hrel.back() / hrel[hrel.size() - 2]) <= 10.0 * innerTol;
                else if (!hrel.empty()) near = hrel.back() <= 10.0 * innerTol;
                ahead = j + 1 < m && !near;
                if (ahead) forwardF32Dev(V + (size_t)(j + 1) * n16, W32, s);
                HIP_CHECK(hipEventSynchronize(hs.ev));
                double worst = 0.0;
                for (int c = 0; c < KC; ++c) {
                    if (hs.p[4 * c + 2] != (double)(j + 1))
                        throw std::runtime_error("16-RHS solve: Arnoldi step " + std::to_string(j) + " left no status");
                    worst = std::max(worst, hs.p[4 * c]);
                }
                ++its;
                used = j + 1;
                hrel.push_back(worst);
                if (worst <= innerTol) break;
            }
            arn::k_arn_solve<<<KC, arn::kThreads, arn::solve_lds(used), s>>>(m, used, st, sts);
            HIP_LAUNCH_CHECK();
            k16_axpy<<<g16, 256, (size_t)used * KC * sizeof(double), s>>>(n16, used, V, n16, st, sts, m, D);
            HIP_LAUNCH_CHECK();
        }
        k16_add<<<g16, 256, 0, s>>>(n16, D, Xt);
        HIP_LAUNCH_CHECK();
        inner += its;
    }
    k16_scatter<<<g16, 256, 0, s>>>(N, perm, Xt, X, ldx);
    HIP_LAUNCH_CHECK();
    HIP_CHECK(hipStreamSynchronize(s));
    checkDeviceErrors();
    if (outerOut) *outerOut = outer;
    return inner;
}

// the same on host pointers (the MEX shim's 'solve' op): one staging copy each way
int Operator::blockSolveHost(const double* rhs, double* x, int restart, double tol, int maxit, double* hist,
                             int maxhist, double* relres) {
    ensureDevice();
    const size_t bytes = (size_t)ks * geo.N * sizeof(double);
    DevBuf db, dx;
    db.alloc(bytes);
    dx.alloc(bytes);
    HIP_CHECK(hipMemcpyAsync(db.p, rhs, bytes, hipMemcpyHostToDevice, own));
    HIP_CHECK(hipMemcpyAsync(dx.p, x, bytes, hipMemcpyHostToDevice, own));
    const int it = blockSolveDev(db.as<double>(), dx.as<double>(), restart, tol, maxit, hist, maxhist, relres, own);
    HIP_CHECK(hipMemcpyAsync(x, dx.p, bytes, hipMemcpyDeviceToHost, own));
    HIP_CHECK(hipStreamSynchronize(own));
    return it;
}

}  // namespace aniso
