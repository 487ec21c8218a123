/*
 * AnisoWrapperMI355X.c -- the reference-side binding of the MI355X matvec: a
 * MATLAB MEX plugin with the op set of AnisoWrapper.mexa64 (AnisoWrapper.cpp:10-136,
 * dispatched by mexplus MEX_DISPATCH, AnisoWrapper.h:15 / dispatch.h:302-317) over
 * the C ABI of libaniso_mi355x.so (include/aniso_mi355x.h), plus the block operator
 * of aniso.m (aniso.m:121-157) as three more ops.
 *
 *   mex -R2018a AnisoWrapperMI355X.c -I<repo>/include -L<repo>/aniso_amd -laniso_mi355x
 *
 * MATLAB usage is unchanged from the reference (Aniso.m / aniso.m):
 *   h = AnisoWrapperMI355X('new', sz, d, ks, g, ns, np, maxLevel);
 *   AnisoWrapperMI355X('setCoeff', h, sigma_s, sigma_t);  AnisoWrapperMI355X('cache', h, id);
 *   theta = AnisoWrapperMI355X('mapping', h, charge, id);
 * and aniso.m's GMRES operator (aniso.m:155) becomes one call per matvec:
 *   A = @(x) AnisoWrapperMI355X('blockMatvec', h, x);   % x - mforward(x), x = [u_0; ...; u_{ks-1}]
 * and aniso.m:159-173's solve, gmres(A, rhs, 400, 1e-11, 400), as one call with the
 * Krylov basis resident on the GPU:
 *   [u, relres, iters] = AnisoWrapperMI355X('solve', h, rhs, 400, 1e-11, 400);
 *
 * MATLAB is absent from this image and from the GPU box: tests/test_integration.py
 * compiles this file for syntax against a declaration-only mex.h (tests/mex_stub).
 */
#include <stdint.h>
#include <string.h>

#include "aniso_mi355x.h"
#include "mex.h"

static void fail(int rc) {
    char msg[1024];
    aniso_last_error(msg, sizeof msg);
    mexErrMsgIdAndTxt(rc == ANISO_ERR_HANDLE ? "mexplus:session:notFound" : "mexplus:arguments:error", "%s", msg);
}

#define CALL(x)               \
    do {                      \
        int rc__ = (x);       \
        if (rc__) fail(rc__); \
    } while (0)

static void need(int nrhs, int n, const char* op) {
    if (nrhs < n) mexErrMsgIdAndTxt("mexplus:arguments:error", "%s: expected %d arguments", op, n - 1);
}

/* the handle travels as an int64 scalar, as Session<Aniso>::create returned it
 * (dispatch.h:189-195, mxINT64_CLASS via mxtypes.h:150-155) */
static aniso_handle handle_of(const mxArray* a) {
    if (!mxIsInt64(a) || mxGetNumberOfElements(a) != 1)
        mexErrMsgIdAndTxt("mexplus:session:invalidType", "handle must be an int64 scalar");
    return (aniso_handle)(intptr_t)(*(const int64_t*)mxGetData(a));
}

static int64_t num_nodes(aniso_handle h) {
    int64_t n = 0;
    CALL(aniso_num_nodes(h, &n));
    return n;
}

static int64_t num_blocks(aniso_handle h) {
    int ks = 0;
    CALL(aniso_num_blocks(h, &ks));
    return ks;
}

/* a real double vector of exactly n entries (the reference's asserts were compiled
 * out, AnisoWrapper.cpp:55-56; this shim checks) */
static const double* column(const mxArray* a, int64_t n, const char* what) {
    if (!mxIsDouble(a) || mxIsComplex(a) || (int64_t)mxGetNumberOfElements(a) != n)
        mexErrMsgIdAndTxt("mexplus:arguments:error", "%s must be a real double vector of %lld entries", what,
                          (long long)n);
    return mxGetPr(a);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char op[32];
    if (nrhs < 1 || mxGetString(prhs[0], op, sizeof op))
        mexErrMsgIdAndTxt("mexplus:dispatch:argumentError", "first argument must be the operation name");
    if (!strcmp(op, "new")) { /* AnisoWrapper.cpp:10-25: (sz, d, ks, g, ns, np, maxLevel) */
        aniso_handle h = NULL;
        need(nrhs, 8, op);
        CALL(aniso_create((int)mxGetScalar(prhs[1]), (int)mxGetScalar(prhs[2]), (int)mxGetScalar(prhs[3]),
                          mxGetScalar(prhs[4]), (int)mxGetScalar(prhs[5]), (int)mxGetScalar(prhs[6]),
                          (int)mxGetScalar(prhs[7]), &h));
        plhs[0] = mxCreateNumericMatrix(1, 1, mxINT64_CLASS, mxREAL);
        *(int64_t*)mxGetData(plhs[0]) = (int64_t)(intptr_t)h;
        mexLock(); /* the plugin stays loaded while a handle lives (dispatch.h:189-195) */
    } else if (!strcmp(op, "delete")) { /* :27-31 */
        need(nrhs, 2, op);
        CALL(aniso_destroy(handle_of(prhs[1])));
        mexUnlock();
    } else if (!strcmp(op, "getNodes")) { /* :33-44, N x 2 column-major */
        aniso_handle h;
        need(nrhs, 2, op);
        h = handle_of(prhs[1]);
        plhs[0] = mxCreateDoubleMatrix((size_t)num_nodes(h), 2, mxREAL);
        CALL(aniso_get_nodes(h, mxGetPr(plhs[0])));
    } else if (!strcmp(op, "setCoeff")) { /* :46-69 */
        aniso_handle h;
        int64_t n;
        need(nrhs, 4, op);
        h = handle_of(prhs[1]);
        n = num_nodes(h);
        CALL(aniso_set_coeff(h, column(prhs[2], n, "sigma_s"), column(prhs[3], n, "sigma_t")));
    } else if (!strcmp(op, "cache")) { /* :72-90 */
        need(nrhs, 3, op);
        CALL(aniso_cache(handle_of(prhs[1]), (int)mxGetScalar(prhs[2])));
    } else if (!strcmp(op, "mapping")) { /* :92-136 */
        aniso_handle h;
        int64_t n;
        need(nrhs, 4, op);
        h = handle_of(prhs[1]);
        n = num_nodes(h);
        plhs[0] = mxCreateDoubleMatrix((size_t)n, 1, mxREAL);
        CALL(aniso_mapping(h, column(prhs[2], n, "charge"), (int)mxGetScalar(prhs[3]), mxGetPr(plhs[0])));
    } else if (!strcmp(op, "forward") || !strcmp(op, "mforward") || !strcmp(op, "blockMatvec")) {
        /* aniso.m:121-136 forward, :138-157 mforward, :155 x - mforward(x); the
         * argument is the stacked column [u_0; ...; u_{ks-1}] of ks * N entries */
        aniso_handle h;
        int64_t len;
        const double* u;
        const int which = !strcmp(op, "forward") ? 0 : !strcmp(op, "mforward") ? 1 : 2;
        need(nrhs, 3, op);
        h = handle_of(prhs[1]);
        /* the library reads and writes exactly ks * N doubles */
        len = num_blocks(h) * num_nodes(h);
        u = column(prhs[2], len, "u"); /* the stacked column [u_0; ...; u_{ks-1}], exactly ks * N */
        plhs[0] = mxCreateDoubleMatrix((size_t)len, 1, mxREAL);
        CALL(aniso_block_op(h, which, u, mxGetPr(plhs[0])));
    } else if (!strcmp(op, "solve")) {
        /* aniso.m:159-173 in one call: [u, relres, iters] = ('solve', h, rhs, restart, tol, maxit)
         * = gmres(@(x) x - mforward(x), rhs, restart, tol, maxit) with every Krylov
         * vector in HBM (MATLAB's call: restart 400, tol 1e-11, maxit 400) */
        aniso_handle h;
        int64_t len;
        const double* rhs;
        int iters = 0;
        double relres = 0.0;
        need(nrhs, 6, op);
        h = handle_of(prhs[1]);
        len = num_blocks(h) * num_nodes(h);
        rhs = column(prhs[2], len, "rhs");
        plhs[0] = mxCreateDoubleMatrix((size_t)len, 1, mxREAL); /* zeros: MATLAB's default x0 */
        CALL(aniso_block_solve(h, rhs, mxGetPr(plhs[0]), (int)mxGetScalar(prhs[3]), mxGetScalar(prhs[4]),
                               (int)mxGetScalar(prhs[5]), NULL, 0, &iters, &relres));
        if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(relres);
        if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)iters);
    } else {
        mexErrMsgIdAndTxt("mexplus:dispatch:argumentError", "Unknown operation %s", op);
    }
}
