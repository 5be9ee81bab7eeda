/* Stub of the MATLAB MEX C API subset used by krylov_robustness_amd/mex/
 * kt_mex.cpp (TEST INFRASTRUCTURE ONLY).  MATLAB is not installed: the CPU
 * suite type-checks the shim against this header, and mex_runtime.cpp
 * implements it so that the GPU suite can run the shim's mexFunction
 * (tests/test_mex_exec.py).  As in MATLAB's own mex.h, mexFunction has C
 * linkage. */
#pragma once
#include <stddef.h>
typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;
typedef enum { mxREAL = 0, mxCOMPLEX } mxComplexity;
extern "C" {
bool mxIsDouble(const mxArray*);
bool mxIsComplex(const mxArray*);
bool mxIsSparse(const mxArray*);
bool mxIsEmpty(const mxArray*);
bool mxIsChar(const mxArray*);
mwSize mxGetM(const mxArray*);
mwSize mxGetN(const mxArray*);
mwIndex* mxGetJc(const mxArray*);
mwIndex* mxGetIr(const mxArray*);
double* mxGetDoubles(const mxArray*);
double mxGetScalar(const mxArray*);
int mxGetString(const mxArray*, char*, mwSize);
mxArray* mxCreateDoubleMatrix(mwSize, mwSize, mxComplexity);
mxArray* mxCreateDoubleScalar(double);
mxArray* mxCreateSparse(mwSize, mwSize, mwSize, mxComplexity);
double mxGetInf(void);
double mxGetNaN(void);
void mxDestroyArray(mxArray*);
int mexCallMATLAB(int, mxArray**, int, mxArray**, const char*);
bool mxIsClass(const mxArray*, const char*);
bool mxIsCell(const mxArray*);
bool mxIsStruct(const mxArray*);
size_t mxGetNumberOfElements(const mxArray*);
mxArray* mxGetCell(const mxArray*, mwIndex);
mxArray* mxGetField(const mxArray*, mwIndex, const char*);
int mexPrintf(const char*, ...);
void mexErrMsgIdAndTxt(const char*, const char*, ...);
void mexWarnMsgIdAndTxt(const char*, const char*, ...);
int mexAtExit(void (*)(void));
void mexLock(void);
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);
}
