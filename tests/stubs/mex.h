/* Minimal declarations of the MathWorks MEX/matrix C API used by mex/fmcw_mex.c,
 * for a syntax/type check of the gateway where MATLAB is not installed
 * (tests/test_host.py::test_mex_gateway_compiles).  Signatures follow the
 * documented R2018a interleaved-complex API; nothing here is linked or run. */
#ifndef FMCW_TEST_STUB_MEX_H
#define FMCW_TEST_STUB_MEX_H
#include <stddef.h>
#include <stdint.h>
typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;
typedef enum { mxSINGLE_CLASS = 7, mxINT32_CLASS = 12 } mxClassID;
typedef struct { float real, imag; } mxComplexSingle;
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));
void mexLock(void);
void mexUnlock(void);
int mxGetString(const mxArray* a, char* buf, mwSize n);
double mxGetScalar(const mxArray* a);
mxArray* mxGetField(const mxArray* s, mwSize i, const char* name);
int mxIsStruct(const mxArray* a);
int mxIsNumeric(const mxArray* a);
int mxIsSingle(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsDouble(const mxArray* a);
double* mxGetDoubles(const mxArray* a);
mwSize mxGetNumberOfElements(const mxArray* a);
mwSize mxGetNumberOfDimensions(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
float* mxGetSingles(const mxArray* a);
int32_t* mxGetInt32s(const mxArray* a);
mxComplexSingle* mxGetComplexSingles(const mxArray* a);
mxArray* mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID c, mxComplexity x);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity x);
int mxIsChar(const mxArray* a);
int mxIsInt32(const mxArray* a);
int mxGetNumberOfFields(const mxArray* s);
mxArray* mxGetFieldByNumber(const mxArray* s, mwSize i, int k);
const char* mxGetFieldNameByNumber(const mxArray* s, int k);
char* mxArrayToUTF8String(const mxArray* a);
void* mxGetData(const mxArray* a);
mwSize mxGetM(const mxArray* a);
mwSize mxGetN(const mxArray* a);
void* mxCalloc(mwSize n, mwSize size);
#endif
