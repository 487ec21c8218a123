// solver.hip -- the callers of the hot path: main.cpp's
// forwardOperator u - K_0(sigma_s .* u) (main.cpp:125-136) and the restarted
// GMRES(m) that drives it (gmres.cpp:53-169), with every vector resident in HBM.
// BLAS-1 reductions use a fixed two-level tree so results are deterministic.
#include <hip/hip_runtime.h>

#include <cmath>
#include <stdexcept>
#include <vector>

#include "aniso_op.hpp"
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

}  // namespace aniso
