/* TEST-ONLY stand-in for MATLAB's mex.h / matrix.h (R2018a interleaved-complex
 * API subset used by channel-estimation_amd/matlab/dsce_mex.c).  MATLAB is not
 * in this image; this header lets tests/test_mex_gateway.py compile the
 * gateway and drive its argument checking on the CPU under AddressSanitizer.
 * It is not a MATLAB build and ships nowhere. */
#ifndef DSCE_TEST_MEX_H
#define DSCE_TEST_MEX_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

typedef size_t mwSize;
typedef bool mxLogical;
typedef enum { mxDOUBLE_CLASS, mxINT64_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS } mxClassID;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;
typedef struct { double real, imag; } mxComplexDouble;
typedef struct mxArray_tag {
    mxClassID cls;
    int cplx;
    size_t m, n;
    void* data;
    char* str;
} mxArray;

int mxGetString(const mxArray* a, char* buf, mwSize len);
double mxGetScalar(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
double* mxGetDoubles(const mxArray* a);
mxComplexDouble* mxGetComplexDoubles(const mxArray* a);
mxLogical* mxGetLogicals(const mxArray* a);
int64_t* mxGetInt64s(const mxArray* a);
bool mxIsComplex(const mxArray* a);
bool mxIsDouble(const mxArray* a);
bool mxIsNumeric(const mxArray* a);
bool mxIsLogical(const mxArray* a);
bool mxIsChar(const mxArray* a);
mxArray* mxDuplicateArray(const mxArray* a);
int mxMakeArrayComplex(mxArray* a);
void mxDestroyArray(mxArray* a);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity c);
void* mxMalloc(size_t n);
void mxFree(void* p);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));
void mexLock(void);
void mexUnlock(void);
#endif
