/*
 * oracle.h -- CPU restatement of the lowrank/aniso reference matvec.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline.  The product (aniso_amd/) never
 * links or calls it.
 *
 * Parity status: the reference is NOT buildable in this image (bbfmm/utils.h:27
 * includes <cblas.h>, which the image lacks; gmres.h:21 also collides with
 * std::abs).  The restatement is pinned by (a) the reference's own Gauss-Legendre
 * tables (tests/golden/gauss_legendre_ref.json, bit-exact), (b) tree/list/pair
 * counts and apply known-answers recorded by the survey's probe of the reference
 * (tests/golden/survey_known_answers.json).  See DESIGN.md "Oracle".
 */
#ifndef ANISO_ORACLE_H
#define ANISO_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle oracle_t;
typedef struct otree otree_t;

/* Aniso(sz, d, ks, g, ns, np, maxLevel)  -- Aniso.cpp:7-13, KernelFactory.cpp:7-54 */
oracle_t *oracle_create(int sz, int d, int ks, double g, int ns, int np, int maxLevel);
void oracle_destroy(oracle_t *o);
int64_t oracle_num_nodes(oracle_t *o);
/* getNodes: N x 2 column-major (AnisoWrapper.cpp:33-44) */
void oracle_get_nodes(oracle_t *o, double *xy);
void oracle_get_weights(oracle_t *o, double *w);
/* setCoeff (AnisoWrapper.cpp:46-69) */
void oracle_set_coeff(oracle_t *o, const double *sigma_s, const double *sigma_t);
/* cache(Id) (AnisoWrapper.cpp:72-90) */
void oracle_cache(oracle_t *o, int id);
/* free mode id's caches (not in the reference: bounds the full-size CPU leg's memory) */
void oracle_uncache(oracle_t *o, int id);
/* mapping(charge, Id) (AnisoWrapper.cpp:92-136); out: N doubles */
void oracle_mapping(oracle_t *o, const double *charge, int id, double *out);
/* Same apply, split by stage; stages is 6*N:
 *   [0] imag FMM   (runKernelsFast)           [1] real FMM (runKernelsFastSing)
 *   [2] nearRemoval contribution (negative)   [3] refineAddOnFast
 *   [4] singularAddFast                        [5] final output (sum * 1/(2 pi))  */
void oracle_mapping_stages(oracle_t *o, const double *charge, int id, double *stages);
/* rebuild the FMM trees on every apply like the reference (default 1) */
void oracle_set_faithful_rebuild(oracle_t *o, int on);
/* timing mode: the reference's per-use heap vectors and block copies (results unchanged) */
void oracle_set_reference_alloc(oracle_t *o, int on);
/* main.cpp:125-141: GMRES(m, maxit, tol) on u - K_0(sigma_s .* u) = K_0 q.
 * x (N) in: initial guess, out: solution.  hist receives up to maxhist residuals.
 * returns the iteration count j at exit (negative if not converged). */
int oracle_gmres_main(oracle_t *o, const double *q, double *x, int m, int maxit, double tol,
                      double *hist, int maxhist, double *final_resid);
/* internals exported for tests */
int oracle_refine_size(oracle_t *o);
void oracle_get_matrices(oracle_t *o, double *interpolate /* d2*d2 col-major */,
                         double *nearMapping /* 16d2*d2 col-major */, double *legendreNorms /* d2 */,
                         double *sqrtWeights /* d2 */);
double oracle_line_integral(oracle_t *o, double x0, double y0, double x1, double y1);
double oracle_eval_kernel(oracle_t *o, int imag, int mode, double ax, double ay, double bx, double by);

/* ---- standalone tree (bbfmm.h:146-449) ---- */
otree_t *otree_build(const double *x, const double *y, int n, int rank, int maxLevel);
void otree_destroy(otree_t *t);
int otree_num_nodes(otree_t *t);
int otree_max_level(otree_t *t);
/* per node: parent, child[4], level, slot, isLeaf, isEmpty, nSource  (11 ints) */
void otree_node_ints(otree_t *t, int id, int *out11);
/* per node: cx, cy, rx, ry */
void otree_node_geom(otree_t *t, int id, double *out4);
/* list: 0=U 1=V 2=W 3=X ; returns length, copies sorted ids into out (may be NULL) */
int otree_list(otree_t *t, int id, int which, int *out);
/* source indices of node id (ascending); returns count */
int otree_sources(otree_t *t, int id, int *out);

#ifdef __cplusplus
}
#endif
#endif
