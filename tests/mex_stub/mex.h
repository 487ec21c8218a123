/* Declaration-only stand-in for MATLAB's mex.h, used by tests/test_integration.py to
 * syntax-check integration/AnisoWrapperMI355X.c (MATLAB is not in this image).  It
 * declares the subset of the MEX API the shim uses, with MATLAB's signatures; it is
 * never linked or run. */
#ifndef ANISO_TEST_MEX_STUB_H
#define ANISO_TEST_MEX_STUB_H
#include <stddef.h>
typedef struct mxArray_tag mxArray;
typedef enum { mxREAL = 0, mxCOMPLEX } mxComplexity;
typedef enum { mxUNKNOWN_CLASS = 0, mxDOUBLE_CLASS = 6, mxINT64_CLASS = 14 } mxClassID;
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
void mexLock(void);
void mexUnlock(void);
int mxGetString(const mxArray* a, char* buf, size_t len);
void* mxGetData(const mxArray* a);
double* mxGetPr(const mxArray* a);
double mxGetScalar(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
int mxIsInt64(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsComplex(const mxArray* a);
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID c, mxComplexity f);
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity f);
mxArray* mxCreateDoubleScalar(double v);
#endif
