// host_geometry.cpp -- quadrature geometry and the small per-mode correction
// tables.  Restates Geometry.cpp:10-154 and KernelFactory.cpp:7-54, 863-986;
// the correction tables re-express KernelFactory.cpp:445-478, 662-709, 828-860
// as translation-invariant stencils (DESIGN.md "Corrections").
#include <cmath>
#include <stdexcept>

#include "gauss_legendre_table.h"
#include "host.hpp"

namespace aniso {

// std::tr1::legendre (libstdc++ tr1/legendre_function.tcc __poly_legendre_p)
double legendre_tr1(unsigned l, double x) {
    if (x == 1.0) return 1.0;
    if (x == -1.0) return (l % 2 == 1) ? -1.0 : 1.0;
    double p_lm2 = 1.0;
    if (l == 0) return p_lm2;
    double p_lm1 = x;
    if (l == 1) return p_lm1;
    double p_l = 0.0;
    for (unsigned ll = 2; ll <= l; ++ll) {
        p_l = 2.0 * x * p_lm1 - p_lm2 - (x * p_lm1 - p_lm2) / (double)ll;
        p_lm2 = p_lm1;
        p_lm1 = p_l;
    }
    return p_l;
}

// get_legendre_data (Quadrature.cpp:5418-22191), regenerated bit-exactly by tools/gen_gauss.py
void gauss_rule(int deg, double* x, double* w) {
    if (deg < 1 || deg > ANISO_GAUSS_MAX_DEG)
        throw std::invalid_argument("quadrature degree " + std::to_string(deg) + " is not implemented (1.." +
                                    std::to_string(ANISO_GAUSS_MAX_DEG) + ")");
    int off = aniso_gauss_off[deg - 1];
    for (int i = 0; i < deg; ++i) {
        x[i] = aniso_gauss_x[off + i];
        w[i] = aniso_gauss_w[off + i];
    }
}

// makeLegendreMatrix (Geometry.cpp:129-154), K rows x cols col-major
static void legendre_matrix(std::vector<double>& K, int rows, int cols, int N, const std::vector<double>& x,
                            const std::vector<double>& y, const std::vector<double>& w, std::vector<double>& norms) {
    K.assign((size_t)rows * cols, 0.0);
    int row = 0;
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < N; ++k) {
            for (int I = 0; I < cols; ++I)
                K[row + (size_t)I * rows] = legendre_tr1(n, x[I]) * legendre_tr1(k, y[I]) * std::sqrt(w[I]);
            ++row;
        }
    norms.assign(rows, 0.0);
    for (row = 0; row < rows; ++row) {
        double nrm = 0.0;
        for (int c = 0; c < cols; ++c) nrm += K[row + (size_t)c * rows] * K[row + (size_t)c * rows];
        nrm = std::sqrt(nrm);
        norms[row] = nrm;
        for (int c = 0; c < cols; ++c) K[row + (size_t)c * rows] /= nrm;
    }
}

void Geometry::build(int sz_, int d_, int ns_) {
    if (sz_ < 1) throw std::invalid_argument("domain size must be >= 1");
    sz = sz_;
    d = d_;
    d2 = d * d;
    ns = ns_;
    gx.resize(d);
    gw.resize(d);
    gauss_rule(d, gx.data(), gw.data());
    dx = 1.0 / sz;
    nsq = sz * sz;
    N = (int64_t)nsq * d2;
    if (N > (int64_t)1 << 30) throw std::invalid_argument("too many quadrature points");
    qx.resize(d2); qy.resize(d2); qw.resize(d2); sqrtW.resize(d2);
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) {
            qx[r * d + c] = gx[r];
            qy[r * d + c] = gx[c];
            qw[r * d + c] = gw[r] * gw[c];
            sqrtW[r * d + c] = std::sqrt(qw[r * d + c]);
        }
    px.resize(N); py.resize(N); w.resize(N);
    for (int i = 0; i < sz; ++i)
        for (int j = 0; j < sz; ++j)
            for (int k = 0; k < d2; ++k) {
                size_t id = (size_t)(i * sz + j) * d2 + k;
                px[id] = (0.5 + i) * dx + 0.5 * (qx[k]) * dx;
                py[id] = (0.5 + j) * dx + 0.5 * qy[k] * dx;
                w[id] = qw[k] * 0.25 * (dx * dx);
            }
    std::vector<double> norms;
    legendre_matrix(interp, d2, d2, d, qx, qy, qw, norms);
    // two-level refinement (Geometry.cpp:69-107)
    refx = qx; refy = qy; refw = qw;
    nref = d2;
    for (int level = 0; level < 2; ++level) {
        std::vector<double> tx, ty, tw;
        for (int id = 0; id < nref; ++id) {
            tx.push_back((refx[id] + 1) / 2.0); ty.push_back((refy[id] + 1) / 2.0); tw.push_back(refw[id] / 4.0);
            tx.push_back((refx[id] + 1) / 2.0); ty.push_back((refy[id] - 1) / 2.0); tw.push_back(refw[id] / 4.0);
            tx.push_back((refx[id] - 1) / 2.0); ty.push_back((refy[id] + 1) / 2.0); tw.push_back(refw[id] / 4.0);
            tx.push_back((refx[id] - 1) / 2.0); ty.push_back((refy[id] - 1) / 2.0); tw.push_back(refw[id] / 4.0);
        }
        refx.swap(tx); refy.swap(ty); refw.swap(tw);
        nref *= 4;
    }
    std::vector<double> refinements;
    legendre_matrix(refinements, d2, nref, d, refx, refy, refw, lnorm);  // quirk: norms of refinements
    nearMap.assign((size_t)nref * d2, 0.0);
    for (int r = 0; r < nref; ++r)
        for (int c = 0; c < d2; ++c) {
            double s = 0.0;
            for (int k = 0; k < d2; ++k) s += refinements[k + (size_t)r * d2] * interp[k + (size_t)c * d2];
            nearMap[r + (size_t)c * nref] = s;
        }
    // singular rule + Duffy precompute (KernelFactory.cpp:15-16, 863-986)
    sgx.resize(ns); sgw.resize(ns);
    gauss_rule(ns, sgx.data(), sgw.data());
    for (int k = 0; k < ns; ++k) {
        sgw[k] /= 2.0;
        sgx[k] += 1.0;
        sgx[k] /= 2.0;
    }
    int ns2 = ns * ns;
    nsing = 8 * ns2;
    singX.assign((size_t)d2 * nsing, 0.0);
    singY.assign((size_t)d2 * nsing, 0.0);
    singW.assign((size_t)d2 * nsing, 0.0);
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) {
            int tid = r * d + c;
            double x = gx[r], y = gx[c];
            const double tri[8][6] = {{x, y, 1., y, 1., 1.},    {x, y, 1., 1, x, 1.},     {x, y, x, 1., -1., 1.},
                                      {x, y, -1., 1., -1., y},  {x, y, -1., y, -1., -1.}, {x, y, -1., -1, x, -1.},
                                      {x, y, x, -1., 1., -1.}, {x, y, 1., -1, 1., y}};
            for (int t = 0; t < 8; ++t) {
                const double* pt = tri[t];
                double a = pt[0], b = pt[1];
                double a11 = pt[2] - pt[0], a12 = pt[4] - pt[2], a21 = pt[3] - pt[1], a22 = pt[5] - pt[3];
                double detA = a11 * a22 - a12 * a21;
                int id = 0;
                for (int ri = 0; ri < ns; ++ri)
                    for (int ci = 0; ci < ns; ++ci) {
                        double u = sgx[ri], v = sgx[ci], ww = sgw[ri] * sgw[ci];
                        double z1x = u, z1y = u * v, z1w = ww * u;
                        size_t o = (size_t)tid * nsing + t * ns2 + id;
                        singX[o] = a11 * z1x + a12 * z1y + a;
                        singY[o] = a21 * z1x + a22 * z1y + b;
                        singW[o] = detA * z1w;
                        ++id;
                    }
            }
        }
}

// real part of the pair kernel, makeKernels (KernelFactory.cpp:243-253); (ax,ay) = source - target
static double real_kernel(int m, double ax, double ay) {
    double dist = std::sqrt(ax * ax + ay * ay);
    if (dist == 0.) return 0.;
    if (m == 0) return 1.0 / dist;
    return std::cos(m * std::atan2(ay, ax)) / dist;
}

void CorrTables::build(const Geometry& g, int m) {
    const int d = g.d, d2 = g.d2, nref = g.nref;
    const double dx = g.dx;
    // 3x3 stencil: C[tq][q9][c], q9 = (dr+1)*3 + (dc+1); dr shifts x (square index i), dc shifts y (j).
    C.assign((size_t)d2 * 9 * d2, 0.0);
    std::vector<double> kr(nref);
    for (int tq = 0; tq < d2; ++tq)
        for (int dr = -1; dr <= 1; ++dr)
            for (int dc = -1; dc <= 1; ++dc) {
                int q9 = (dr + 1) * 3 + (dc + 1);
                double* row = &C[((size_t)tq * 9 + q9) * d2];
                // nearRemoval: - real(x_s - x_t) for every coarse source point (self included)
                for (int c = 0; c < d2; ++c) {
                    double ax = (dr + 0.5 * (g.qx[c] - g.qx[tq])) * dx;
                    double ay = (dc + 0.5 * (g.qy[c] - g.qy[tq])) * dx;
                    row[c] = -real_kernel(m, ax, ay);
                }
                if (dr == 0 && dc == 0) continue;
                // refineAddOn: sum_r real(p_r - x_t) sqrt(w_r) nearMapping(r,c) / sqrtW(c)
                for (int r = 0; r < nref; ++r) {
                    double ax = (dr + 0.5 * (g.refx[r] - g.qx[tq])) * dx;
                    double ay = (dc + 0.5 * (g.refy[r] - g.qy[tq])) * dx;
                    kr[r] = real_kernel(m, ax, ay) * std::sqrt(g.refw[r]);
                }
                for (int c = 0; c < d2; ++c) {
                    double s = 0.0;
                    for (int r = 0; r < nref; ++r) s += kr[r] * g.nearMap[r + (size_t)c * nref];
                    row[c] += s / g.sqrtW[c];
                }
            }
    // singular moments mu[tq][a][b] = sum_p (h u_p)^a (h v_p)^b S[tq][p]
    const double h = 0.5 * dx;
    mu.assign((size_t)d2 * d * d, 0.0);
    for (int tq = 0; tq < d2; ++tq)
        for (int p = 0; p < g.nsing; ++p) {
            size_t o = (size_t)tq * g.nsing + p;
            double ax = 0.5 * (g.singX[o] - g.qx[tq]) * dx;
            double ay = 0.5 * (g.singY[o] - g.qy[tq]) * dx;
            double S = real_kernel(m, ax, ay) * (g.singW[o] * (dx * dx) / 4.0);
            double ua = 1.0;
            for (int a = 0; a < d; ++a) {
                double vb = 1.0;
                for (int b = 0; b < d; ++b) {
                    mu[((size_t)tq * d + a) * d + b] += ua * vb * S;
                    vb *= h * g.singY[o];
                }
                ua *= h * g.singX[o];
            }
        }
    // Legendre monomial coefficients L[n][e] and Taylor-shift table
    // legB[(n*d + a)*d + e'] = L[n][a+e'] * binom(a+e', a), so that
    // P_n(X + s) = sum_a s^a sum_e' legB[n][a][e'] X^e'.
    std::vector<double> L((size_t)d * d, 0.0);
    L[0] = 1.0;
    if (d > 1) L[1 * d + 1] = 1.0;
    for (int n = 1; n + 1 < d; ++n)
        for (int e = 0; e < d; ++e) {
            double v = -(double)n * L[(n - 1) * d + e];
            if (e > 0) v += (2.0 * n + 1.0) * L[n * d + e - 1];
            L[(n + 1) * d + e] = v / (n + 1.0);
        }
    legB.assign((size_t)d * d * d, 0.0);
    for (int n = 0; n < d; ++n)
        for (int a = 0; a <= n; ++a)
            for (int e = a; e <= n; ++e) {
                double binom = 1.0;
                for (int k = 1; k <= a; ++k) binom = binom * (e - a + k) / k;
                legB[((size_t)n * d + a) * d + (e - a)] = L[n * d + e] * binom;
            }
    coefScale.resize(d2);
    for (int k = 0; k < d2; ++k) coefScale[k] = 1.0 / g.lnorm[k];
}

}  // namespace aniso
