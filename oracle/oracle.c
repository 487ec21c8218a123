/*
 * oracle.c -- plain-C restatement of the lowrank/aniso reference matvec
 * (`mapping(charge, Id)`, AnisoWrapper.cpp:92-136) and everything it depends on.
 *
 * TEST INFRASTRUCTURE ONLY -- see oracle.h.  It is the checker for the HIP product
 * path and the timed CPU baseline ("kind": "port") in bench.py; the product never
 * calls it.  Every function cites the reference file:line it restates.  Structure
 * deliberately follows the reference (recursive tree, per-node cached operator
 * matrices, per-target correction loops, tree rebuilt on every apply) so that its
 * timing is a faithful CPU baseline; lists are kept as sorted sets instead of
 * std::unordered_set, which changes summation order only.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../aniso_amd/csrc/gauss_legendre_table.h"

#define EPS 1e-12 /* bbfmm/utils.h:46 */
#define SQR(x) ((x) * (x))

/* ------------------------------------------------------------------ helpers */

typedef struct {
    int n, cap;
    int *a;
} ivec;

static void iv_push(ivec *v, int x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 8;
        v->a = (int *)realloc(v->a, sizeof(int) * v->cap);
    }
    v->a[v->n++] = x;
}

/* std::unordered_set<int>::insert restated as a sorted set */
static void iv_insert(ivec *v, int x) {
    int lo = 0, hi = v->n;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (v->a[mid] < x) lo = mid + 1; else hi = mid;
    }
    if (lo < v->n && v->a[lo] == x) return;
    iv_push(v, x);
    memmove(v->a + lo + 1, v->a + lo, sizeof(int) * (v->n - 1 - lo));
    v->a[lo] = x;
}

static void iv_free(ivec *v) { free(v->a); v->a = NULL; v->n = v->cap = 0; }

static void *xcalloc(size_t n, size_t s) {
    void *p = calloc(n ? n : 1, s);
    if (!p) { fprintf(stderr, "oracle: out of memory (%zu x %zu)\n", n, s); abort(); }
    return p;
}

/* std::tr1::legendre (libstdc++ 11 tr1/legendre_function.tcc __poly_legendre_p),
 * used by Geometry.cpp:134 and KernelFactory.cpp:184,202,850 */
static double legendre(unsigned l, double x) {
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

/* get_legendre_data (Quadrature.cpp:5418-22191), table regenerated bit-exactly */
static void gauss_rule(int deg, double *x, double *w) {
    if (deg < 1 || deg > ANISO_GAUSS_MAX_DEG) {
        fprintf(stderr, "oracle: quadrature degree %d not supported\n", deg);
        abort();
    }
    int off = aniso_gauss_off[deg - 1];
    for (int i = 0; i < deg; ++i) { x[i] = aniso_gauss_x[off + i]; w[i] = aniso_gauss_w[off + i]; }
}

/* ===================================================================== tree
 * bbfmm::tree (bbfmm.h:146-449)
 */
typedef struct {
    int parent, child[4], level, slot;
    double cx, cy, rx, ry;
    int nsrc, srccap;
    int *src;
    int isLeaf, isEmpty;
    ivec U, V, W, X;
} onode;

struct otree {
    onode *nd;
    int nn, cap;
    double *px, *py;
    int n;
    int rank, maxLevelArg, maxLevel;
    double cx, cy, rx, ry;
};

static int tree_new_node(otree_t *t, int level, int slot) {
    if (t->nn == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 64;
        t->nd = (onode *)realloc(t->nd, sizeof(onode) * t->cap);
    }
    onode *n = &t->nd[t->nn];
    memset(n, 0, sizeof(*n));
    n->parent = -1;
    for (int i = 0; i < 4; ++i) n->child[i] = -1;
    n->level = level;
    n->slot = slot;
    return t->nn++;
}

static void node_push_src(onode *n, int idx) {
    if (n->nsrc == n->srccap) {
        n->srccap = n->srccap ? 2 * n->srccap : 16;
        n->src = (int *)realloc(n->src, sizeof(int) * n->srccap);
    }
    n->src[n->nsrc++] = idx;
}

/* assignChildren (bbfmm.h:250-317) */
static void tree_assign_children(otree_t *t, int id) {
    if (t->nd[id].nsrc == 0) {
        t->nd[id].isLeaf = 1;
        t->nd[id].isEmpty = 1;
        return;
    }
    if (t->nd[id].nsrc <= t->rank || t->nd[id].level == t->maxLevelArg) {
        t->nd[id].isLeaf = 1;
        if (t->maxLevel < t->nd[id].level) t->maxLevel = t->nd[id].level;
        return;
    }
    for (int i = 0; i < 4; ++i) {
        int c = tree_new_node(t, t->nd[id].level + 1, i);
        onode *p = &t->nd[id];
        onode *ch = &t->nd[c];
        p->child[i] = c;
        ch->parent = id;
        ch->cx = p->cx + ((i & 1) - 0.5) * p->rx;
        ch->cy = p->cy + (((i >> 1) & 1) - 0.5) * p->ry;
        ch->rx = p->rx * 0.5;
        ch->ry = p->ry * 0.5;
    }
    onode *p = &t->nd[id];
    for (int k = 0; k < p->nsrc; ++k) {
        int idx = p->src[k];
        int y_bit = t->py[idx] < p->cy ? 0 : 1;
        int x_bit = t->px[idx] < p->cx ? 0 : 1;
        node_push_src(&t->nd[p->child[2 * y_bit + x_bit]], idx);
    }
    for (int i = 0; i < 4; ++i) tree_assign_children(t, t->nd[id].child[i]);
}

/* findNode (bbfmm.h:416-429) */
static int tree_find(otree_t *t, double x, double y) {
    int id = 0;
    for (;;) {
        onode *n = &t->nd[id];
        if (fabs(n->cx - x) < EPS && fabs(n->cy - y) < EPS) return id;
        if (n->isLeaf) return id;
        int x_bit = n->cx > x ? 0 : 1;
        int y_bit = n->cy > y ? 0 : 1;
        id = n->child[2 * y_bit + x_bit];
    }
}

/* isAdjacent (bbfmm.h:431-447) */
static int tree_adjacent(otree_t *t, int a, int b) {
    onode *A = &t->nd[a], *B = &t->nd[b];
    double diff_x = fabs(A->cx - B->cx), diff_y = fabs(A->cy - B->cy);
    double r_x = fabs(A->rx + B->rx), r_y = fabs(A->ry + B->ry);
    int rdx = r_x >= diff_x - EPS;
    int rdy = r_y >= diff_y - EPS;
    int x_adj = (fabs(diff_x - r_x) < EPS) && rdy;
    int y_adj = (fabs(diff_y - r_y) < EPS) && rdx;
    return x_adj || y_adj;
}

/* buildNode (bbfmm.h:334-413) */
static void tree_build_node(otree_t *t, int id, double minx, double miny, double maxx, double maxy) {
    onode *n = &t->nd[id];
    iv_free(&n->U); iv_free(&n->V); iv_free(&n->W); iv_free(&n->X);
    if (n->parent != -1) {
        onode *pn = &t->nd[n->parent];
        double dx = n->rx, dy = n->ry;
        double xs = pn->cx - dx, ys = pn->cy - dy;
        int qcap = 64, *queue = (int *)malloc(sizeof(int) * qcap);
        for (int x_id = -2; x_id < 4; x_id++) {
            for (int y_id = -2; y_id < 4; y_id++) {
                double curx = xs + 2 * x_id * dx;
                double cury = ys + 2 * y_id * dy;
                int le = (curx <= maxx + EPS) && (cury <= maxy + EPS);
                int ge = (curx >= minx - EPS) && (cury >= miny - EPS);
                int eq = fabs(curx - n->cx) < EPS && fabs(cury - n->cy) < EPS;
                if (!(le && ge && !eq)) continue;
                int curId = tree_find(t, curx, cury);
                int adj = tree_adjacent(t, id, curId);
                onode *cn = &t->nd[curId];
                if (cn->level < n->level) {
                    if (adj) {
                        if (cn->isLeaf) iv_insert(&n->U, curId);
                    } else {
                        iv_insert(&n->X, curId);
                    }
                }
                if (cn->level == n->level) {
                    if (!adj) {
                        iv_insert(&n->V, curId);
                    } else if (n->isLeaf) {
                        int head = 0, tail = 0;
                        queue[tail++] = curId;
                        while (head < tail) {
                            int f = queue[head++];
                            onode *fn = &t->nd[f];
                            if (!tree_adjacent(t, f, id)) {
                                iv_insert(&n->W, f);
                            } else if (fn->isLeaf) {
                                iv_insert(&n->U, f);
                            } else {
                                if (tail + 4 > qcap) {
                                    qcap *= 2;
                                    queue = (int *)realloc(queue, sizeof(int) * qcap);
                                }
                                for (int i = 0; i < 4; ++i) queue[tail++] = fn->child[i];
                            }
                        }
                    }
                }
            }
        }
        free(queue);
    }
    if (n->isLeaf) iv_insert(&n->U, id);
}

/* populate + getCenterRadius (bbfmm.h:176-209, 231-248) */
otree_t *otree_build(const double *x, const double *y, int n, int rank, int maxLevel) {
    otree_t *t = (otree_t *)xcalloc(1, sizeof(otree_t));
    t->n = n;
    t->px = (double *)xcalloc(n, sizeof(double));
    t->py = (double *)xcalloc(n, sizeof(double));
    memcpy(t->px, x, sizeof(double) * n);
    memcpy(t->py, y, sizeof(double) * n);
    t->rank = rank;
    t->maxLevelArg = maxLevel;
    t->maxLevel = 0;
    double x_max = x[0], x_min = x[0], y_max = y[0], y_min = y[0];
    for (int i = 0; i < n; ++i) {
        x_max = fmax(x_max, x[i]); y_max = fmax(y_max, y[i]);
        x_min = fmin(x_min, x[i]); y_min = fmin(y_min, y[i]);
    }
    t->cx = (x_max + x_min) / 2.0;
    t->cy = (y_max + y_min) / 2.0;
    t->rx = (x_max - x_min) / 2.0;
    t->ry = (y_max - y_min) / 2.0;
    int root = tree_new_node(t, 0, 0);
    t->nd[root].cx = t->cx; t->nd[root].cy = t->cy;
    t->nd[root].rx = t->rx; t->nd[root].ry = t->ry;
    for (int i = 0; i < n; ++i) node_push_src(&t->nd[root], i);
    tree_assign_children(t, root);
    double minx = t->cx - t->rx, miny = t->cy - t->ry, maxx = t->cx + t->rx, maxy = t->cy + t->ry;
    int nn = t->nn;
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < nn; ++i) tree_build_node(t, i, minx, miny, maxx, maxy);
    return t;
}

void otree_destroy(otree_t *t) {
    if (!t) return;
    for (int i = 0; i < t->nn; ++i) {
        onode *n = &t->nd[i];
        free(n->src);
        iv_free(&n->U); iv_free(&n->V); iv_free(&n->W); iv_free(&n->X);
    }
    free(t->nd); free(t->px); free(t->py); free(t);
}

int otree_num_nodes(otree_t *t) { return t->nn; }
int otree_max_level(otree_t *t) { return t->maxLevel; }

void otree_node_ints(otree_t *t, int id, int *o) {
    onode *n = &t->nd[id];
    o[0] = n->parent;
    for (int i = 0; i < 4; ++i) o[1 + i] = n->child[i];
    o[5] = n->level; o[6] = n->slot; o[7] = n->isLeaf; o[8] = n->isEmpty; o[9] = n->nsrc; o[10] = 0;
}

void otree_node_geom(otree_t *t, int id, double *o) {
    onode *n = &t->nd[id];
    o[0] = n->cx; o[1] = n->cy; o[2] = n->rx; o[3] = n->ry;
}

int otree_list(otree_t *t, int id, int which, int *out) {
    onode *n = &t->nd[id];
    ivec *v = which == 0 ? &n->U : which == 1 ? &n->V : which == 2 ? &n->W : &n->X;
    if (out) memcpy(out, v->a, sizeof(int) * v->n);
    return v->n;
}

int otree_sources(otree_t *t, int id, int *out) {
    onode *n = &t->nd[id];
    if (out) memcpy(out, n->src, sizeof(int) * n->nsrc);
    return n->nsrc;
}

/* ================================================================ operator */

typedef struct {
    otree_t *t;
    int imag, mode, np, rank;
    double *cheb;   /* np */
    double *tnode;  /* np x np col-major, tnode(i,l) = T_l(c_i) */
    double *R[4];   /* rank x rank col-major */
    double **cache; /* per node: V,X,U,W matrices (non-empty sources), col-major */
    double *nodeCharge, *nodePotential; /* nn x rank */
    int built;
} fmm_t;

struct oracle {
    int sz, d, d2, ks, kernelSize, ns, np, maxLevel;
    double g, dx;
    int nsq, N;
    double *px, *py, *w;
    double *gx, *gw;
    double *qx, *qy, *qw, *sqrtW;
    int nref;
    double *refx, *refy, *refw;
    double *interp;  /* d2 x d2 col-major */
    double *nearMap; /* nref x d2 col-major */
    double *lnorm;   /* d2 */
    double *sgx, *sgw;
    int nsing;
    double *sigma_s, *sigma_t, *st_coeff, *ss_coeff;
    double *singX, *singY, *singW; /* d2 x nsing */
    fmm_t *imag, *real;
    double **nearI; /* [mode] N*9*nref */
    double **singI; /* [mode] N*nsing */
    int faithful;
    int refalloc; /* timing mode: the reference's per-use heap vectors (oracle_set_reference_alloc) */
};

/* makeLegendreMatrix (Geometry.cpp:129-154); K is rows x cols col-major */
static void make_legendre_matrix(double *K, int rows, int cols, int N, const double *x, const double *y,
                                 const double *w, double *norms) {
    int row = 0;
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < N; ++k) {
            for (int I = 0; I < cols; ++I)
                K[row + (size_t)I * rows] = legendre(n, x[I]) * legendre(k, y[I]) * sqrt(w[I]);
            ++row;
        }
    for (row = 0; row < rows; ++row) {
        double nrm = 0.0;
        for (int c = 0; c < cols; ++c) nrm += SQR(K[row + (size_t)c * rows]);
        nrm = sqrt(nrm);
        norms[row] = nrm;
        for (int c = 0; c < cols; ++c) K[row + (size_t)c * rows] /= nrm;
    }
}

/* Geometry::Geometry (Geometry.cpp:10-114) + KernelFactory ctor (KernelFactory.cpp:7-54) */
oracle_t *oracle_create(int sz, int d, int ks, double g, int ns, int np, int maxLevel) {
    oracle_t *o = (oracle_t *)xcalloc(1, sizeof(oracle_t));
    o->sz = sz; o->d = d; o->d2 = d * d; o->ks = ks; o->kernelSize = 2 * ks - 1;
    o->ns = ns; o->np = np; o->maxLevel = maxLevel; o->g = g;
    o->faithful = 1;
    o->dx = 1.0 / sz;
    o->nsq = sz * sz;
    o->N = o->nsq * o->d2;
    int d2 = o->d2;
    o->gx = (double *)xcalloc(d, sizeof(double));
    o->gw = (double *)xcalloc(d, sizeof(double));
    gauss_rule(d, o->gx, o->gw);
    o->qx = (double *)xcalloc(d2, sizeof(double));
    o->qy = (double *)xcalloc(d2, sizeof(double));
    o->qw = (double *)xcalloc(d2, sizeof(double));
    o->sqrtW = (double *)xcalloc(d2, sizeof(double));
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) {
            o->qx[r * d + c] = o->gx[r];
            o->qy[r * d + c] = o->gx[c];
            o->qw[r * d + c] = o->gw[r] * o->gw[c];
            o->sqrtW[r * d + c] = sqrt(o->qw[r * d + c]);
        }
    o->px = (double *)xcalloc(o->N, sizeof(double));
    o->py = (double *)xcalloc(o->N, sizeof(double));
    o->w = (double *)xcalloc(o->N, sizeof(double));
    double dx = o->dx;
    for (int i = 0; i < sz; ++i)
        for (int j = 0; j < sz; ++j)
            for (int k = 0; k < d2; ++k) {
                size_t id = (size_t)(i * sz + j) * d2 + k;
                o->px[id] = (0.5 + i) * dx + 0.5 * (o->qx[k]) * dx;
                o->py[id] = (0.5 + j) * dx + 0.5 * o->qy[k] * dx;
                o->w[id] = o->qw[k] * 0.25 * SQR(dx);
            }
    o->lnorm = (double *)xcalloc(d2, sizeof(double));
    o->interp = (double *)xcalloc((size_t)d2 * d2, sizeof(double));
    make_legendre_matrix(o->interp, d2, d2, d, o->qx, o->qy, o->qw, o->lnorm);
    /* two-level refinement rule (Geometry.cpp:69-107) */
    int nref = d2;
    double *rx = (double *)xcalloc(nref, sizeof(double)), *ry = (double *)xcalloc(nref, sizeof(double)),
           *rw = (double *)xcalloc(nref, sizeof(double));
    memcpy(rx, o->qx, sizeof(double) * d2);
    memcpy(ry, o->qy, sizeof(double) * d2);
    memcpy(rw, o->qw, sizeof(double) * d2);
    for (int level = 0; level < 2; ++level) {
        double *tx = (double *)xcalloc(4 * nref, sizeof(double)), *ty = (double *)xcalloc(4 * nref, sizeof(double)),
               *tw = (double *)xcalloc(4 * nref, sizeof(double));
        int m = 0;
        for (int id = 0; id < nref; ++id) {
            tx[m] = (rx[id] + 1) / 2.0; ty[m] = (ry[id] + 1) / 2.0; tw[m++] = rw[id] / 4.0;
            tx[m] = (rx[id] + 1) / 2.0; ty[m] = (ry[id] - 1) / 2.0; tw[m++] = rw[id] / 4.0;
            tx[m] = (rx[id] - 1) / 2.0; ty[m] = (ry[id] + 1) / 2.0; tw[m++] = rw[id] / 4.0;
            tx[m] = (rx[id] - 1) / 2.0; ty[m] = (ry[id] - 1) / 2.0; tw[m++] = rw[id] / 4.0;
        }
        free(rx); free(ry); free(rw);
        rx = tx; ry = ty; rw = tw;
        nref *= 4;
    }
    o->nref = nref;
    o->refx = rx; o->refy = ry; o->refw = rw;
    double *refinements = (double *)xcalloc((size_t)d2 * nref, sizeof(double));
    make_legendre_matrix(refinements, d2, nref, d, rx, ry, rw, o->lnorm); /* quirk: norms overwritten */
    o->nearMap = (double *)xcalloc((size_t)nref * d2, sizeof(double));
    for (int r = 0; r < nref; ++r)
        for (int c = 0; c < d2; ++c) {
            double s = 0.0;
            for (int k = 0; k < d2; ++k) s += refinements[k + (size_t)r * d2] * o->interp[k + (size_t)c * d2];
            o->nearMap[r + (size_t)c * nref] = s;
        }
    free(refinements);
    /* singular rule: get_legendre_data(ns) + affine (KernelFactory.cpp:15-16, Quadrature.cpp:22194-22200) */
    o->sgx = (double *)xcalloc(ns, sizeof(double));
    o->sgw = (double *)xcalloc(ns, sizeof(double));
    gauss_rule(ns, o->sgx, o->sgw);
    for (int k = 0; k < ns; ++k) {
        o->sgw[k] /= 2.0;
        o->sgx[k] += 1.0;
        o->sgx[k] /= 2.0;
    }
    o->nsing = 8 * ns * ns;
    o->sigma_s = (double *)xcalloc(o->N, sizeof(double));
    o->sigma_t = (double *)xcalloc(o->N, sizeof(double));
    o->st_coeff = (double *)xcalloc((size_t)o->nsq * d2, sizeof(double));
    o->ss_coeff = (double *)xcalloc((size_t)o->nsq * d2, sizeof(double));
    o->imag = (fmm_t *)xcalloc(o->kernelSize, sizeof(fmm_t));
    o->real = (fmm_t *)xcalloc(o->kernelSize, sizeof(fmm_t));
    o->nearI = (double **)xcalloc(o->kernelSize, sizeof(double *));
    o->singI = (double **)xcalloc(o->kernelSize, sizeof(double *));
    return o;
}

static void fmm_free(fmm_t *f) {
    if (f->t) {
        if (f->cache) {
            for (int i = 0; i < f->t->nn; ++i) free(f->cache[i]);
            free(f->cache);
        }
        otree_destroy(f->t);
    }
    free(f->cheb); free(f->tnode);
    for (int i = 0; i < 4; ++i) free(f->R[i]);
    free(f->nodeCharge); free(f->nodePotential);
    memset(f, 0, sizeof(*f));
}

void oracle_destroy(oracle_t *o) {
    if (!o) return;
    for (int i = 0; i < o->kernelSize; ++i) {
        fmm_free(&o->imag[i]); fmm_free(&o->real[i]);
        free(o->nearI[i]); free(o->singI[i]);
    }
    free(o->imag); free(o->real); free(o->nearI); free(o->singI);
    free(o->px); free(o->py); free(o->w); free(o->gx); free(o->gw);
    free(o->qx); free(o->qy); free(o->qw); free(o->sqrtW);
    free(o->refx); free(o->refy); free(o->refw); free(o->interp); free(o->nearMap); free(o->lnorm);
    free(o->sgx); free(o->sgw); free(o->sigma_s); free(o->sigma_t); free(o->st_coeff); free(o->ss_coeff);
    free(o->singX); free(o->singY); free(o->singW);
    free(o);
}

int64_t oracle_num_nodes(oracle_t *o) { return o->N; }
int oracle_refine_size(oracle_t *o) { return o->nref; }
void oracle_set_faithful_rebuild(oracle_t *o, int on) { o->faithful = on; }
/* Timing mode (results unchanged): repeat the reference's per-use heap traffic on the
 * apply path -- the cached block deep-copied on every use (K = Cache[rootId][cnt],
 * bbfmm.h:1053, Matrix::operator= linalg.h:213-237), the two Vectors per target and
 * neighbour of refineAddOnFast (KernelFactory.cpp:684-685) and the Vector load(d^2) +
 * ddot per Duffy point of singularAddFast (KernelFactory.cpp:847-855). */
void oracle_set_reference_alloc(oracle_t *o, int on) { o->refalloc = on; }

/* the reference's Vector(n): new scalar_t[n] + memset (linalg.h:20-27) */
static double *ref_vector(int n) {
    double *v = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    if (!v) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    memset(v, 0, sizeof(double) * (size_t)n);
    return v;
}
/* cblas_ddot as a call the compiler cannot inline into the loop (blas_wrapper.cpp) */
__attribute__((noinline)) static double ref_ddot(int n, const double *x, const double *y) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += x[i] * y[i];
    return s;
}
/* Matrix::operator= of a cached block (delete[] + new[] + memcpy, linalg.h:213-237) */
static const double *ref_copy(double **held, const double *K, size_t n) {
    free(*held);
    *held = (double *)malloc(sizeof(double) * (n ? n : 1));
    if (!*held) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    memcpy(*held, K, sizeof(double) * n);
    return *held;
}

void oracle_get_nodes(oracle_t *o, double *xy) {
    for (int i = 0; i < o->N; ++i) { xy[i] = o->px[i]; xy[i + o->N] = o->py[i]; }
}

void oracle_get_weights(oracle_t *o, double *w) { memcpy(w, o->w, sizeof(double) * o->N); }

void oracle_get_matrices(oracle_t *o, double *interp, double *nearMap, double *lnorm, double *sqrtW) {
    int d2 = o->d2;
    if (interp) memcpy(interp, o->interp, sizeof(double) * d2 * d2);
    if (nearMap) memcpy(nearMap, o->nearMap, sizeof(double) * (size_t)o->nref * d2);
    if (lnorm) memcpy(lnorm, o->lnorm, sizeof(double) * d2);
    if (sqrtW) memcpy(sqrtW, o->sqrtW, sizeof(double) * d2);
}

/* getRow / getCol (KernelFactory.cpp:392-401) */
static inline int get_row(oracle_t *o, double y) { return (int)floor(y * o->sz); }
static inline int get_col(oracle_t *o, double x) { return (int)floor(x * o->sz); }

/* dgemv(1, interpolate, sqrtW .* h_sq, 0, c) (KernelFactory.cpp:212-227, 988-1005) */
static void interp_square(oracle_t *o, const double *h, double *c) {
    int d2 = o->d2;
    for (int r = 0; r < d2; ++r) {
        double s = 0.0;
        for (int k = 0; k < d2; ++k) s += o->interp[r + (size_t)k * d2] * (o->sqrtW[k] * h[k]);
        c[r] = s;
    }
}

/* integral_helper (KernelFactory.cpp:174-190) -- Legendre at GLOBAL coords (quirk 1) */
static double integral_helper(oracle_t *o, double x0, double y0, double x1, double y1) {
    int d = o->d;
    int col = get_row(o, (x0 + x1) / 2);
    int row = get_col(o, (y0 + y1) / 2);
    const double *coef = o->st_coeff + (size_t)(col * o->sz + row) * o->d2;
    double ret = 0.0;
    for (int i = 0; i < d; ++i) {
        double x = (x0 + x1) / 2 + (x0 - x1) / 2 * o->gx[i];
        double y = (y0 + y1) / 2 + (y0 - y1) / 2 * o->gx[i];
        double dot = 0.0;
        for (int n = 0; n < d; ++n)
            for (int k = 0; k < d; ++k)
                dot += legendre(n, x) * legendre(k, y) / o->lnorm[n * d + k] * coef[n * d + k];
        ret += dot * o->gw[i];
    }
    return ret * sqrt(SQR(x0 - x1) + SQR(y0 - y1)) / 2.0;
}

/* lineIntegral (KernelFactory.cpp:67-166) */
static double line_integral(oracle_t *o, double x0, double y0, double x1, double y1) {
    int col0 = get_row(o, x0), col1 = get_row(o, x1);
    int row0 = get_col(o, y0), row1 = get_col(o, y1);
    double side = 1.0 / o->dx;
    if ((row0 == row1) && (col0 == col1)) return integral_helper(o, x0, y0, x1, y1);
    if ((row0 == row1 + 1) && (col0 == col1)) {
        double ybar = (double)row0 / side;
        double xbar = ((y1 - ybar) * x0 + (ybar - y0) * x1) / (y1 - y0);
        return integral_helper(o, x0, y0, xbar, ybar) + integral_helper(o, xbar, ybar, x1, y1);
    }
    if ((row0 == row1 - 1) && (col0 == col1)) {
        double ybar = (double)row1 / side;
        double xbar = ((y1 - ybar) * x0 + (ybar - y0) * x1) / (y1 - y0);
        return integral_helper(o, x0, y0, xbar, ybar) + integral_helper(o, xbar, ybar, x1, y1);
    }
    if ((col0 == col1 + 1) && (row0 == row1)) {
        double xbar = (double)col0 / side;
        double ybar = ((x1 - xbar) * y0 + (xbar - x0) * y1) / (x1 - x0);
        return integral_helper(o, x0, y0, xbar, ybar) + integral_helper(o, xbar, ybar, x1, y1);
    }
    if ((col0 == col1 - 1) && (row0 == row1)) {
        double xbar = (double)col1 / side;
        double ybar = ((x1 - xbar) * y0 + (xbar - x0) * y1) / (x1 - x0);
        return integral_helper(o, x0, y0, xbar, ybar) + integral_helper(o, xbar, ybar, x1, y1);
    }
    int diag = 0;
    double xbar = 0, ybar2 = 0;
    if ((col0 == col1 + 1) && (row0 == row1 + 1)) { diag = 1; xbar = (double)col0 / side; ybar2 = (double)row0 / side; }
    else if ((col0 == col1 + 1) && (row0 == row1 - 1)) { diag = 1; xbar = (double)col0 / side; ybar2 = (double)row1 / side; }
    else if ((col0 == col1 - 1) && (row0 == row1 + 1)) { diag = 2; xbar = (double)col1 / side; ybar2 = (double)row0 / side; }
    else if ((col0 == col1 - 1) && (row0 == row1 - 1)) { diag = 2; xbar = (double)col1 / side; ybar2 = (double)row1 / side; }
    if (diag) {
        double ybar = ((x1 - xbar) * y0 + (xbar - x0) * y1) / (x1 - x0);
        double xbar2 = ((y1 - ybar2) * x0 + (ybar2 - y0) * x1) / (y1 - y0);
        int first = diag == 1 ? (xbar < xbar2) : (xbar > xbar2);
        if (first)
            return integral_helper(o, x1, y1, xbar, ybar) + integral_helper(o, xbar, ybar, xbar2, ybar2) +
                   integral_helper(o, xbar2, ybar2, x0, y0);
        return integral_helper(o, x1, y1, xbar2, ybar2) + integral_helper(o, xbar, ybar, xbar2, ybar2) +
               integral_helper(o, xbar, ybar, x0, y0);
    }
    double xm = (x0 + x1) / 2, ym = (y0 + y1) / 2;
    return line_integral(o, x0, y0, xm, ym) + line_integral(o, xm, ym, x1, y1);
}

double oracle_line_integral(oracle_t *o, double x0, double y0, double x1, double y1) {
    return line_integral(o, x0, y0, x1, y1);
}

/* evaluate (KernelFactory.cpp:193-207) */
static double evaluate(oracle_t *o, double px, double py) {
    int d = o->d;
    int col = get_row(o, px), row = get_col(o, py);
    const double *coef = o->st_coeff + (size_t)(col * o->sz + row) * o->d2;
    double s = 0.0;
    for (int n = 0; n < d; ++n)
        for (int k = 0; k < d; ++k) s += legendre(n, px) * legendre(k, py) / o->lnorm[n * d + k] * coef[n * d + k];
    return s;
}

/* makeKernels (KernelFactory.cpp:240-267): a = source, b = target */
static inline double eval_real(int i, double ax, double ay, double bx, double by) {
    double dist = sqrt(SQR(ax - bx) + SQR(ay - by));
    double ang = atan2(ay - by, ax - bx);
    if (i == 0) return dist == 0. ? 0. : 1.0 / dist;
    return dist == 0. ? 0. : cos(i * ang) / dist;
}

static inline double eval_imag(oracle_t *o, int i, double ax, double ay, double bx, double by) {
    double dist = sqrt(SQR(ax - bx) + SQR(ay - by));
    double ang = atan2(ay - by, ax - bx);
    if (i == 0) return dist == 0. ? evaluate(o, ax, ay) : (exp(-line_integral(o, ax, ay, bx, by)) - 1) / dist;
    return dist == 0. ? 0. : (exp(-line_integral(o, ax, ay, bx, by)) - 1) * cos(i * ang) / dist;
}

double oracle_eval_kernel(oracle_t *o, int imag, int mode, double ax, double ay, double bx, double by) {
    return imag ? eval_imag(o, mode, ax, ay, bx, by) : eval_real(mode, ax, ay, bx, by);
}

static inline double fmm_eval(oracle_t *o, fmm_t *f, double ax, double ay, double bx, double by) {
    return f->imag ? eval_imag(o, f->mode, ax, ay, bx, by) : eval_real(f->mode, ax, ay, bx, by);
}

/* setCoeff: copy + interpolation() + singPrecompute() (AnisoWrapper.cpp:46-69) */
static void duffy_transform(oracle_t *o, const double *pt, double *X, double *Y, double *W) {
    /* duffy_transform (KernelFactory.cpp:863-927) */
    double a = pt[0], b = pt[1];
    double a11 = pt[2] - pt[0], a12 = pt[4] - pt[2], a21 = pt[3] - pt[1], a22 = pt[5] - pt[3];
    double detA = a11 * a22 - a12 * a21;
    int nsp = o->ns, id = 0;
    for (int ri = 0; ri < nsp; ++ri)
        for (int ci = 0; ci < nsp; ++ci) {
            double u = o->sgx[ri], v = o->sgx[ci], w = o->sgw[ri] * o->sgw[ci];
            double z1x = u, z1y = u * v, z1w = w * u;
            X[id] = a11 * z1x + a12 * z1y + a;
            Y[id] = a21 * z1x + a22 * z1y + b;
            W[id] = detA * z1w;
            ++id;
        }
}

static void sing_precompute(oracle_t *o) {
    /* singPrecompute (KernelFactory.cpp:929-986) */
    int d = o->d, ns2 = o->ns * o->ns;
    free(o->singX); free(o->singY); free(o->singW);
    o->singX = (double *)xcalloc((size_t)o->d2 * o->nsing, sizeof(double));
    o->singY = (double *)xcalloc((size_t)o->d2 * o->nsing, sizeof(double));
    o->singW = (double *)xcalloc((size_t)o->d2 * o->nsing, sizeof(double));
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) {
            int tid = r * d + c;
            double x = o->gx[r], y = o->gx[c];
            double tri[8][6] = {{x, y, 1., y, 1., 1.},    {x, y, 1., 1, x, 1.},   {x, y, x, 1., -1., 1.},
                                {x, y, -1., 1., -1., y},  {x, y, -1., y, -1., -1.}, {x, y, -1., -1, x, -1.},
                                {x, y, x, -1., 1., -1.}, {x, y, 1., -1, 1., y}};
            for (int t = 0; t < 8; ++t)
                duffy_transform(o, tri[t], o->singX + (size_t)tid * o->nsing + t * ns2,
                                o->singY + (size_t)tid * o->nsing + t * ns2, o->singW + (size_t)tid * o->nsing + t * ns2);
        }
}

void oracle_set_coeff(oracle_t *o, const double *sigma_s, const double *sigma_t) {
    memcpy(o->sigma_s, sigma_s, sizeof(double) * o->N);
    memcpy(o->sigma_t, sigma_t, sizeof(double) * o->N);
    int nsq = o->nsq, d2 = o->d2;
#pragma omp parallel for schedule(static, 80)
    for (int i = 0; i < nsq; ++i) {
        interp_square(o, o->sigma_t + (size_t)i * d2, o->st_coeff + (size_t)i * d2);
        interp_square(o, o->sigma_s + (size_t)i * d2, o->ss_coeff + (size_t)i * d2);
    }
    sing_precompute(o);
}

/* ---------------------------------------------------------------- bbfmm kernel
 * kernel::initialize and Chebyshev operators (bbfmm.h:476-505, 597-693)
 */
static void cheby_poly(int npoly, int n, const double *x, double *T /* n x npoly col-major */) {
    /* getStandardChebyPoly (bbfmm.h:607-630) */
    for (int i = 0; i < n; ++i) T[i] = 1.0;
    if (npoly > 1) {
        for (int i = 0; i < n; ++i) T[i + n] = x[i];
        for (int l = 2; l < npoly; ++l)
            for (int i = 0; i < n; ++i) T[i + (size_t)l * n] = 2.0 * x[i] * T[i + (size_t)(l - 1) * n] - T[i + (size_t)(l - 2) * n];
    }
}

/* S(k,i) = (-1 + 2 sum_l T_l(s_k) T_l(c_i)) / np   (bbfmm.h:635-656, 737-748) */
static void cheby_interp(fmm_t *f, int n, const double *s, double *S /* n x np col-major */) {
    int np = f->np;
    double *T = (double *)xcalloc((size_t)n * np, sizeof(double));
    cheby_poly(np, n, s, T);
    for (int k = 0; k < n; ++k)
        for (int i = 0; i < np; ++i) {
            double acc = 0.0;
            for (int l = 0; l < np; ++l) acc += T[k + (size_t)l * n] * f->tnode[i + l * np];
            S[k + (size_t)i * n] = (2.0 * acc - 1.0) * (1.0 / np);
        }
    free(T);
}

static void fmm_init(oracle_t *o, fmm_t *f, int imag, int mode) {
    /* initialize (bbfmm.h:476-505): tree, Chebyshev nodes, transfer matrices */
    int np = o->np;
    f->imag = imag; f->mode = mode; f->np = np; f->rank = np * np;
    f->t = otree_build(o->px, o->py, o->N, np * np, o->maxLevel);
    f->cheb = (double *)xcalloc(np, sizeof(double));
    for (int i = 0; i < np; ++i) f->cheb[i] = -cos((i + 0.5) * M_PI / np);
    f->tnode = (double *)xcalloc(np * np, sizeof(double));
    cheby_poly(np, np, f->cheb, f->tnode);
    double *child = (double *)xcalloc(2 * np, sizeof(double));
    for (int i = 0; i < np; ++i) { child[i] = -0.5 + 0.5 * f->cheb[i]; child[i + np] = 0.5 + 0.5 * f->cheb[i]; }
    double *S = (double *)xcalloc(2 * np * np, sizeof(double));
    cheby_interp(f, 2 * np, child, S);
    int rk = f->rank;
    for (int id = 0; id < 4; ++id) {
        f->R[id] = (double *)xcalloc((size_t)rk * rk, sizeof(double));
        int b0 = id & 1, b1 = (id >> 1) & 1;
        for (int i = 0; i < np; ++i)
            for (int j = 0; j < np; ++j)
                for (int k = 0; k < np; ++k)
                    for (int l = 0; l < np; ++l)
                        f->R[id][(i * np + j) + (size_t)(k * np + l) * rk] =
                            S[(b1 * np + i) + (size_t)k * 2 * np] * S[(b0 * np + j) + (size_t)l * 2 * np];
    }
    free(child); free(S);
    f->nodeCharge = (double *)xcalloc((size_t)f->t->nn * rk, sizeof(double));
    f->nodePotential = (double *)xcalloc((size_t)f->t->nn * rk, sizeof(double));
    f->built = 1;
}

/* getTransferParentToChildren (bbfmm.h:723-759): R(k, j*np+i) = Sx(k,i) Sy(k,j) */
static void leaf_transfer(fmm_t *f, onode *n, const double *px, const double *py, double *R /* nsrc x rank */) {
    int N = n->nsrc, np = f->np;
    double *sx = (double *)xcalloc(N, sizeof(double)), *sy = (double *)xcalloc(N, sizeof(double));
    for (int i = 0; i < N; ++i) {
        sx[i] = (px[n->src[i]] - n->cx) / n->rx;
        sy[i] = (py[n->src[i]] - n->cy) / n->ry;
    }
    double *Sx = (double *)xcalloc((size_t)N * np, sizeof(double)), *Sy = (double *)xcalloc((size_t)N * np, sizeof(double));
    cheby_interp(f, N, sx, Sx);
    cheby_interp(f, N, sy, Sy);
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < np; ++i)
            for (int j = 0; j < np; ++j) R[k + (size_t)(j * np + i) * N] = Sx[k + (size_t)i * N] * Sy[k + (size_t)j * N];
    free(sx); free(sy); free(Sx); free(Sy);
}

/* Chebyshev points of a node: p = j*np + i <-> (cx + rx c_i, cy + ry c_j)  (bbfmm.h:699-705, 782-804) */
static void cheb_points(fmm_t *f, onode *n, double *x, double *y) {
    int np = f->np;
    for (int j = 0; j < np; ++j)
        for (int i = 0; i < np; ++i) {
            x[j * np + i] = n->cx + n->rx * f->cheb[i];
            y[j * np + i] = n->cy + n->ry * f->cheb[j];
        }
}

/* upPass (bbfmm.h:825-861), level by level instead of OMP tasks */
static void fmm_up(oracle_t *o, fmm_t *f, const double *charge) {
    otree_t *t = f->t;
    int rk = f->rank;
    memset(f->nodeCharge, 0, sizeof(double) * (size_t)t->nn * rk);
    for (int L = t->maxLevel; L >= 0; --L) {
#pragma omp parallel for schedule(dynamic, 16)
        for (int id = 0; id < t->nn; ++id) {
            onode *n = &t->nd[id];
            if (n->level != L) continue;
            double *nc = f->nodeCharge + (size_t)id * rk;
            if (n->isLeaf) {
                if (n->nsrc == 0) continue;
                double *R = (double *)xcalloc((size_t)n->nsrc * rk, sizeof(double));
                leaf_transfer(f, n, t->px, t->py, R);
                for (int c = 0; c < rk; ++c) {
                    double s = 0.0;
                    for (int k = 0; k < n->nsrc; ++k) s += R[k + (size_t)c * n->nsrc] * charge[n->src[k]];
                    nc[c] += s;
                }
                free(R);
            } else {
                for (int i = 0; i < 4; ++i) {
                    onode *ch = &t->nd[n->child[i]];
                    if (ch->isEmpty) continue;
                    const double *cc = f->nodeCharge + (size_t)n->child[i] * rk;
                    for (int c = 0; c < rk; ++c) {
                        double s = 0.0;
                        for (int r = 0; r < rk; ++r) s += f->R[i][r + (size_t)c * rk] * cc[r];
                        nc[c] += s;
                    }
                }
            }
        }
    }
    (void)o;
}

/* number of matrices and doubles cached for node id (downPassCache order V,X,U,W) */
static size_t node_cache_size(fmm_t *f, int id) {
    otree_t *t = f->t;
    onode *n = &t->nd[id];
    size_t sz = 0;
    int rk = f->rank;
    if (n->parent != -1) {
        for (int k = 0; k < n->V.n; ++k) if (!t->nd[n->V.a[k]].isEmpty) sz += (size_t)rk * rk;
        for (int k = 0; k < n->X.n; ++k) if (!t->nd[n->X.a[k]].isEmpty) sz += (size_t)rk * rk;
    }
    if (n->isLeaf && n->nsrc != 0) {
        for (int k = 0; k < n->U.n; ++k) { onode *s = &t->nd[n->U.a[k]]; if (!s->isEmpty) sz += (size_t)n->nsrc * s->nsrc; }
        for (int k = 0; k < n->W.n; ++k) { onode *s = &t->nd[n->W.a[k]]; if (!s->isEmpty) sz += (size_t)n->nsrc * s->nsrc; }
    }
    return sz;
}

/* downPassCache (bbfmm.h:949-1039): evaluate every pair operator once and store it */
static void fmm_build_cache(oracle_t *o, fmm_t *f) {
    otree_t *t = f->t;
    int rk = f->rank;
    f->cache = (double **)xcalloc(t->nn, sizeof(double *));
#pragma omp parallel for schedule(dynamic, 4)
    for (int id = 0; id < t->nn; ++id) {
        onode *n = &t->nd[id];
        size_t sz = node_cache_size(f, id);
        if (!sz) continue;
        double *buf = (double *)xcalloc(sz, sizeof(double));
        f->cache[id] = buf;
        double tx[64], ty[64], sx[64], sy[64];
        if (n->parent != -1) {
            cheb_points(f, n, tx, ty);
            for (int pass = 0; pass < 2; ++pass) {
                ivec *lst = pass == 0 ? &n->V : &n->X;
                for (int k = 0; k < lst->n; ++k) {
                    onode *s = &t->nd[lst->a[k]];
                    if (s->isEmpty) continue;
                    cheb_points(f, s, sx, sy);
                    for (int b = 0; b < rk; ++b)
                        for (int a = 0; a < rk; ++a) buf[a + (size_t)b * rk] = fmm_eval(o, f, sx[b], sy[b], tx[a], ty[a]);
                    buf += (size_t)rk * rk;
                }
            }
        }
        if (n->isLeaf && n->nsrc != 0) {
            for (int pass = 0; pass < 2; ++pass) {
                ivec *lst = pass == 0 ? &n->U : &n->W;
                for (int k = 0; k < lst->n; ++k) {
                    onode *s = &t->nd[lst->a[k]];
                    if (s->isEmpty) continue;
                    for (int b = 0; b < s->nsrc; ++b)
                        for (int a = 0; a < n->nsrc; ++a)
                            buf[a + (size_t)b * n->nsrc] =
                                fmm_eval(o, f, t->px[s->src[b]], t->py[s->src[b]], t->px[n->src[a]], t->py[n->src[a]]);
                    buf += (size_t)n->nsrc * s->nsrc;
                }
            }
        }
    }
}

/* downPassFast (bbfmm.h:1041-1129), level by level (parents before children) */
static void fmm_down(oracle_t *o, fmm_t *f, const double *charge, double *potential) {
    otree_t *t = f->t;
    int rk = f->rank;
    memset(f->nodePotential, 0, sizeof(double) * (size_t)t->nn * rk);
    for (int L = 1; L <= t->maxLevel; ++L) {
#pragma omp parallel for schedule(dynamic, 16)
        for (int id = 0; id < t->nn; ++id) {
            onode *n = &t->nd[id];
            if (n->level != L) continue;
            double *np_ = f->nodePotential + (size_t)id * rk;
            const double *K = f->cache[id];
            double *held = NULL;
            for (int pass = 0; pass < 2; ++pass) {
                ivec *lst = pass == 0 ? &n->V : &n->X;
                for (int k = 0; k < lst->n; ++k) {
                    if (t->nd[lst->a[k]].isEmpty) continue;
                    const double *sc = f->nodeCharge + (size_t)lst->a[k] * rk;
                    const double *Ku = o->refalloc ? ref_copy(&held, K, (size_t)rk * rk) : K;
                    for (int a = 0; a < rk; ++a) {
                        double s = 0.0;
                        for (int b = 0; b < rk; ++b) s += Ku[a + (size_t)b * rk] * sc[b];
                        np_[a] += s;
                    }
                    K += (size_t)rk * rk;
                }
            }
            free(held);
            const double *pp = f->nodePotential + (size_t)n->parent * rk;
            for (int a = 0; a < rk; ++a) {
                double s = 0.0;
                for (int b = 0; b < rk; ++b) s += f->R[n->slot][a + (size_t)b * rk] * pp[b];
                np_[a] += s;
            }
        }
    }
    int nn = t->nn;
#pragma omp parallel for schedule(dynamic, 16)
    for (int id = 0; id < nn; ++id) {
        onode *n = &t->nd[id];
        if (!(n->isLeaf && n->nsrc != 0)) continue;
        /* skip the M2L matrices at the front of this node's cache */
        const double *K = f->cache[id];
        if (n->parent != -1) {
            for (int k = 0; k < n->V.n; ++k) if (!t->nd[n->V.a[k]].isEmpty) K += (size_t)rk * rk;
            for (int k = 0; k < n->X.n; ++k) if (!t->nd[n->X.a[k]].isEmpty) K += (size_t)rk * rk;
        }
        int nT = n->nsrc;
        double *pot = (double *)xcalloc(nT, sizeof(double));
        double *held = NULL;
        for (int pass = 0; pass < 2; ++pass) {
            ivec *lst = pass == 0 ? &n->U : &n->W;
            for (int k = 0; k < lst->n; ++k) {
                onode *s = &t->nd[lst->a[k]];
                if (s->isEmpty) continue;
                const double *Ku = o->refalloc ? ref_copy(&held, K, (size_t)nT * s->nsrc) : K;
                for (int a = 0; a < nT; ++a) {
                    double acc = 0.0;
                    for (int b = 0; b < s->nsrc; ++b) acc += Ku[a + (size_t)b * nT] * charge[s->src[b]];
                    pot[a] += acc;
                }
                K += (size_t)nT * s->nsrc;
            }
        }
        free(held);
        /* L2T: pot += L * nodePotential (L built like R for targets) */
        double *L = (double *)xcalloc((size_t)nT * rk, sizeof(double));
        leaf_transfer(f, n, t->px, t->py, L);
        const double *np_ = f->nodePotential + (size_t)id * rk;
        for (int a = 0; a < nT; ++a) {
            double acc = 0.0;
            for (int c = 0; c < rk; ++c) acc += L[a + (size_t)c * nT] * np_[c];
            pot[a] += acc;
        }
        free(L);
        for (int a = 0; a < nT; ++a) potential[n->src[a]] += pot[a];
        free(pot);
    }
    (void)o;
}

static void fmm_rebuild_tree(oracle_t *o, fmm_t *f) {
    /* kernel::initialize re-populates the tree on every apply (KernelFactory.cpp:356-358) */
    otree_t *nt = otree_build(o->px, o->py, o->N, f->rank, o->maxLevel);
    if (nt->nn != f->t->nn) { fprintf(stderr, "oracle: tree rebuild changed the tree\n"); abort(); }
    otree_t *old = f->t;
    f->t = nt;
    otree_destroy(old);
}

static void fmm_apply(oracle_t *o, fmm_t *f, const double *charge, double *potential) {
    if (o->faithful) fmm_rebuild_tree(o, f);
    memset(potential, 0, sizeof(double) * o->N);
    fmm_up(o, f, charge);
    fmm_down(o, f, charge, potential);
}

/* refineAddOnCache (KernelFactory.cpp:550-609) */
static void refine_cache(oracle_t *o, int mode) {
    int sz = o->sz, d2 = o->d2, nref = o->nref;
    double dx = o->dx;
    free(o->nearI[mode]);
    double *C = (double *)xcalloc((size_t)o->N * 9 * nref, sizeof(double));
    o->nearI[mode] = C;
    int nsq = o->nsq;
#pragma omp parallel for collapse(2) schedule(static, 80)
    for (int tsq = 0; tsq < nsq; ++tsq)
        for (int tq = 0; tq < d2; ++tq) {
            int tid = tsq * d2 + tq;
            int trow = tsq / sz, tcol = tsq - sz * trow;
            for (int dr = -1; dr < 2; ++dr)
                for (int dc = -1; dc < 2; ++dc) {
                    int nsq_ = tsq + dr * sz + dc;
                    if (nsq_ == tsq) continue;
                    if (!(dr + trow >= 0 && dr + trow < sz)) continue;
                    if (!(dc + tcol >= 0 && dc + tcol < sz)) continue;
                    double *dst = C + ((size_t)tid * 9 + (dr + 1) * 3 + (dc + 1)) * nref;
                    for (int r = 0; r < nref; ++r) {
                        double lambda = o->refx[r], mu = o->refy[r], w = o->refw[r];
                        double cx = (0.5 + (trow + dr)) * dx + 0.5 * (lambda)*dx;
                        double cy = (0.5 + (tcol + dc)) * dx + 0.5 * (mu)*dx;
                        dst[r] = eval_real(mode, cx, cy, o->px[tid], o->py[tid]) * sqrt(w);
                    }
                }
        }
}

/* singularAddCache (KernelFactory.cpp:752-788) */
static void sing_cache(oracle_t *o, int mode) {
    int sz = o->sz, d2 = o->d2, ns = o->nsing;
    double dx = o->dx;
    free(o->singI[mode]);
    double *C = (double *)xcalloc((size_t)o->N * ns, sizeof(double));
    o->singI[mode] = C;
    int nsq = o->nsq;
#pragma omp parallel for collapse(2) schedule(static, 80)
    for (int tsq = 0; tsq < nsq; ++tsq)
        for (int tq = 0; tq < d2; ++tq) {
            int col = tsq / sz, row = tsq - col * sz;
            int tid = tsq * d2 + tq;
            for (int p = 0; p < ns; ++p) {
                double x = (0.5 + col) * dx + 0.5 * (o->singX[(size_t)tq * ns + p]) * dx;
                double y = (0.5 + row) * dx + 0.5 * (o->singY[(size_t)tq * ns + p]) * dx;
                double w = o->singW[(size_t)tq * ns + p] * SQR(dx) / 4.0;
                C[(size_t)tid * ns + p] = eval_real(mode, x, y, o->px[tid], o->py[tid]) * w;
            }
        }
}

/* release mode id's caches (the reference keeps every mode cached; the bench's
 * full-size CPU leg caches one mode at a time to bound host memory) */
void oracle_uncache(oracle_t *o, int id) {
    if (id < 0 || id >= o->kernelSize) return;
    fmm_free(&o->imag[id]);
    fmm_free(&o->real[id]);
    free(o->nearI[id]);
    free(o->singI[id]);
    o->nearI[id] = NULL;
    o->singI[id] = NULL;
}

/* cache(Id): runKernelsCache, runKernelsCacheSing, refineAddOnCache, singularAddCache
 * (AnisoWrapper.cpp:72-90, KernelFactory.cpp:279-334) */
void oracle_cache(oracle_t *o, int id) {
    if (id < 0 || id >= o->kernelSize) { fprintf(stderr, "oracle: bad kernel id %d\n", id); abort(); }
    fmm_free(&o->imag[id]);
    fmm_free(&o->real[id]);
    fmm_init(o, &o->imag[id], 1, id);
    fmm_build_cache(o, &o->imag[id]);
    fmm_init(o, &o->real[id], 0, id);
    fmm_build_cache(o, &o->real[id]);
    refine_cache(o, id);
    sing_cache(o, id);
}

/* nearRemoval (KernelFactory.cpp:445-478): ret -= real(s, t) f(s) over 3x3 incl. self */
static void near_removal(oracle_t *o, int mode, const double *f, double *ret) {
    int sz = o->sz, d2 = o->d2, nsq = o->nsq;
#pragma omp parallel for collapse(2) schedule(static, 80)
    for (int tsq = 0; tsq < nsq; ++tsq)
        for (int tq = 0; tq < d2; ++tq) {
            int tid = tsq * d2 + tq;
            int trow = tsq / sz, tcol = tsq - sz * trow;
            for (int dr = -1; dr < 2; ++dr)
                for (int dc = -1; dc < 2; ++dc) {
                    int nsq_ = tsq + dr * sz + dc;
                    if (!(dr + trow >= 0 && dr + trow < sz)) continue;
                    if (!(dc + tcol >= 0 && dc + tcol < sz)) continue;
                    for (int q = 0; q < d2; ++q) {
                        int sid = nsq_ * d2 + q;
                        ret[tid] -= eval_real(mode, o->px[sid], o->py[sid], o->px[tid], o->py[tid]) * f[sid];
                    }
                }
        }
}

/* refineAddOnFast (KernelFactory.cpp:662-709) */
static void refine_fast(oracle_t *o, int mode, const double *f, double *ret) {
    int sz = o->sz, d2 = o->d2, nsq = o->nsq, nref = o->nref;
    const double *C = o->nearI[mode];
#pragma omp parallel for collapse(2) schedule(static, 80)
    for (int tsq = 0; tsq < nsq; ++tsq)
        for (int tq = 0; tq < d2; ++tq) {
            int tid = tsq * d2 + tq;
            int trow = tsq / sz, tcol = tsq - sz * trow;
            double oldv[64], newv[1024];
            for (int dr = -1; dr < 2; ++dr)
                for (int dc = -1; dc < 2; ++dc) {
                    int nsq_ = tsq + dr * sz + dc;
                    if (nsq_ == tsq) continue;
                    if (!(dr + trow >= 0 && dr + trow < sz)) continue;
                    if (!(dc + tcol >= 0 && dc + tcol < sz)) continue;
                    double *ov = oldv, *nv = newv;
                    if (o->refalloc) {  /* Vector oldValues(d^2), newValues(16 d^2) (KernelFactory.cpp:684-685) */
                        ov = ref_vector(d2);
                        nv = ref_vector(nref);
                    }
                    for (int q = 0; q < d2; ++q) ov[q] = f[nsq_ * d2 + q] / o->sqrtW[q];
                    for (int r = 0; r < nref; ++r) {
                        double s = 0.0;
                        for (int c = 0; c < d2; ++c) s += o->nearMap[r + (size_t)c * nref] * ov[c];
                        nv[r] = s;
                    }
                    const double *row = C + ((size_t)tid * 9 + (dr + 1) * 3 + (dc + 1)) * nref;
                    for (int r = 0; r < nref; ++r) ret[tid] += row[r] * nv[r];
                    if (o->refalloc) {
                        free(ov);
                        free(nv);
                    }
                }
        }
}

/* singularAddFast (KernelFactory.cpp:828-860) */
static void singular_fast(oracle_t *o, int mode, const double *coeff, double *ret) {
    int sz = o->sz, d = o->d, d2 = o->d2, nsq = o->nsq, ns = o->nsing;
    double dx = o->dx;
    const double *C = o->singI[mode];
#pragma omp parallel for collapse(2) schedule(static, 80)
    for (int tsq = 0; tsq < nsq; ++tsq)
        for (int tq = 0; tq < d2; ++tq) {
            int col = tsq / sz, row = tsq - col * sz;
            int tid = tsq * d2 + tq;
            const double *cf = coeff + (size_t)(col * sz + row) * d2;
            for (int p = 0; p < ns; ++p) {
                double x = (0.5 + col) * dx + 0.5 * (o->singX[(size_t)tq * ns + p]) * dx;
                double y = (0.5 + row) * dx + 0.5 * (o->singY[(size_t)tq * ns + p]) * dx;
                double dot = 0.0;
                if (o->refalloc) {  /* Vector load(d^2), filled, then ddot (KernelFactory.cpp:847-855) */
                    double *load = ref_vector(d2);
                    for (int n = 0; n < d; ++n)
                        for (int k = 0; k < d; ++k) load[n * d + k] = legendre(n, x) * legendre(k, y) / o->lnorm[n * d + k];
                    dot = ref_ddot(d2, load, cf);
                    free(load);
                } else {
                    for (int n = 0; n < d; ++n)
                        for (int k = 0; k < d; ++k) dot += legendre(n, x) * legendre(k, y) / o->lnorm[n * d + k] * cf[n * d + k];
                }
                ret[tid] += dot * C[(size_t)tid * ns + p];
            }
        }
}

/* mapping (AnisoWrapper.cpp:92-136) */
void oracle_mapping_stages(oracle_t *o, const double *charge, int id, double *st) {
    if (id < 0 || id >= o->kernelSize || !o->imag[id].built) {
        fprintf(stderr, "oracle: mapping on uncached kernel id %d\n", id);
        abort();
    }
    int N = o->N, d2 = o->d2;
    double *fs = (double *)xcalloc(N, sizeof(double));
    double *coef = (double *)xcalloc((size_t)o->nsq * d2, sizeof(double));
    for (int i = 0; i < N; ++i) fs[i] = charge[i] * o->w[i];
    int nsq = o->nsq;
#pragma omp parallel for schedule(static, 80)
    for (int i = 0; i < nsq; ++i) interp_square(o, charge + (size_t)i * d2, coef + (size_t)i * d2);
    double *s_imag = st, *s_real = st + N, *s_rem = st + 2 * (size_t)N, *s_ref = st + 3 * (size_t)N,
           *s_sing = st + 4 * (size_t)N, *s_out = st + 5 * (size_t)N;
    fmm_apply(o, &o->imag[id], fs, s_imag);
    fmm_apply(o, &o->real[id], fs, s_real);
    memset(s_rem, 0, sizeof(double) * N);
    memset(s_ref, 0, sizeof(double) * N);
    memset(s_sing, 0, sizeof(double) * N);
    near_removal(o, id, fs, s_rem);
    refine_fast(o, id, fs, s_ref);
    singular_fast(o, id, coef, s_sing);
    for (int i = 0; i < N; ++i) {
        double out_t = s_real[i] + s_rem[i] + s_ref[i] + s_sing[i];
        out_t += s_imag[i];
        s_out[i] = out_t * (M_1_PI / 2.0);
    }
    free(fs); free(coef);
}

void oracle_mapping(oracle_t *o, const double *charge, int id, double *out) {
    double *st = (double *)xcalloc((size_t)6 * o->N, sizeof(double));
    oracle_mapping_stages(o, charge, id, st);
    memcpy(out, st + 5 * (size_t)o->N, sizeof(double) * o->N);
    free(st);
}

/* ------------------------------------------------------------------ GMRES
 * GMRES(m, max_iter, tol) (gmres.cpp:53-169) driving main.cpp:121-141
 */
static double dnrm2(const double *x, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += x[i] * x[i];
    return sqrt(s);
}

static double ddot(const double *x, const double *y, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += x[i] * y[i];
    return s;
}

static void gen_rot(double dx, double dy, double *cs, double *sn) {
    if (dy == 0.0) { *cs = 1.0; *sn = 0.0; }
    else if (fabs(dy) > fabs(dx)) { double t = dx / dy; *sn = 1.0 / sqrt(1.0 + t * t); *cs = t * *sn; }
    else { double t = dy / dx; *cs = 1.0 / sqrt(1.0 + t * t); *sn = t * *cs; }
}

static void app_rot(double *dx, double *dy, double cs, double sn) {
    double t = cs * *dx + sn * *dy;
    *dy = -sn * *dx + cs * *dy;
    *dx = t;
}

/* forwardOperator (main.cpp:125-136) */
static void forward_op(oracle_t *o, const double *u, double *out, double *tmp) {
    int N = o->N;
    for (int i = 0; i < N; ++i) tmp[i] = u[i] * o->sigma_s[i];
    oracle_mapping(o, tmp, 0, out);
    for (int i = 0; i < N; ++i) out[i] = u[i] - out[i];
}

static void gm_update(double *x, int k, const double *H, int ld, const double *s, double **v, int N) {
    double *y = (double *)xcalloc(k + 1, sizeof(double));
    for (int i = 0; i <= k; ++i) y[i] = s[i];
    for (int i = k; i >= 0; i--) {
        y[i] /= H[i + i * ld];
        for (int j = i - 1; j >= 0; j--) y[j] -= H[j + i * ld] * y[i];
    }
    for (int j = 0; j <= k; j++)
        for (int n = 0; n < N; ++n) x[n] += y[j] * v[j][n];
    free(y);
}

int oracle_gmres_main(oracle_t *o, const double *q, double *x, int m, int maxit, double tol, double *hist,
                      int maxhist, double *final_resid) {
    int N = o->N, nh = 0;
    double *b = (double *)xcalloc(N, sizeof(double)), *r = (double *)xcalloc(N, sizeof(double)),
           *p = (double *)xcalloc(N, sizeof(double)), *tmp = (double *)xcalloc(N, sizeof(double));
    oracle_mapping(o, q, 0, b); /* rhs = apply_mapping(charge) (main.cpp:123) */
    int ld = m + 1, i, j = 1, k, ret = -1;
    double *H = (double *)xcalloc((size_t)ld * ld, sizeof(double));
    double *s = (double *)xcalloc(ld, sizeof(double)), *cs = (double *)xcalloc(ld, sizeof(double)),
           *sn = (double *)xcalloc(ld, sizeof(double));
    double **v = (double **)xcalloc(ld, sizeof(double *));
    for (k = 0; k < ld; ++k) v[k] = (double *)xcalloc(N, sizeof(double));
    double normb = dnrm2(b, N);
    forward_op(o, x, p, tmp);
    for (int n = 0; n < N; ++n) r[n] = b[n] - p[n];
    double beta = dnrm2(r, N), resid;
    if (normb == 0.0) normb = 1;
    if ((resid = dnrm2(r, N) / normb) <= tol) { ret = 0; goto done; }
    while (j <= maxit) {
        for (int n = 0; n < N; ++n) v[0][n] = r[n] * (1.0 / beta);
        memset(s, 0, sizeof(double) * ld);
        s[0] = beta;
        for (i = 0; i < m && j <= maxit; i++, j++) {
            if (hist && nh < maxhist) hist[nh++] = resid;
            forward_op(o, v[i], p, tmp);
            for (k = 0; k <= i; k++) {
                H[k + i * ld] = ddot(p, v[k], N);
                for (int n = 0; n < N; ++n) p[n] -= H[k + i * ld] * v[k][n];
            }
            H[(i + 1) + i * ld] = dnrm2(p, N);
            for (int n = 0; n < N; ++n) v[i + 1][n] = p[n] * (1.0 / H[(i + 1) + i * ld]);
            for (k = 0; k < i; k++) app_rot(&H[k + i * ld], &H[(k + 1) + i * ld], cs[k], sn[k]);
            gen_rot(H[i + i * ld], H[(i + 1) + i * ld], &cs[i], &sn[i]);
            app_rot(&H[i + i * ld], &H[(i + 1) + i * ld], cs[i], sn[i]);
            app_rot(&s[i], &s[i + 1], cs[i], sn[i]);
            if ((resid = fabs(s[i + 1]) / normb) < tol) {
                gm_update(x, i, H, ld, s, v, N);
                ret = j;
                goto done;
            }
        }
        gm_update(x, i - 1, H, ld, s, v, N);
        forward_op(o, x, p, tmp);
        for (int n = 0; n < N; ++n) r[n] = b[n] - p[n];
        beta = dnrm2(r, N);
        if ((resid = beta / normb) < tol) { ret = j; goto done; }
    }
    ret = -j;
done:
    if (final_resid) *final_resid = resid;
    if (hist && nh < maxhist) hist[nh++] = resid;
    for (k = 0; k < ld; ++k) free(v[k]);
    free(v); free(H); free(s); free(cs); free(sn); free(b); free(r); free(p); free(tmp);
    return ret;
}
