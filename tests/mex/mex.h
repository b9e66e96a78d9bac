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

/* MATLAB's two complex storage APIs: R2018a+ (-R2018a) interleaved, R2013b /
 * R2016a separate real / imaginary planes (README.md:19-20).  The test builds
 * the gateway once per API; -DDSCE_TEST_SPLIT selects the split one, and the
 * other API's accessors are then not declared (a gateway that used them would
 * not compile). */
#ifdef DSCE_TEST_SPLIT
#define MX_HAS_INTERLEAVED_COMPLEX 0
#else
#define MX_HAS_INTERLEAVED_COMPLEX 1
#endif

typedef size_t mwSize;
typedef bool mxLogical;
typedef enum { mxDOUBLE_CLASS, mxINT64_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxSTRUCT_CLASS, mxOBJECT_CLASS } mxClassID;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;
typedef struct { double real, imag; } mxComplexDouble;
typedef struct mxArray_tag {
    mxClassID cls;
    int cplx;
    size_t m, n;
    void* data;          /* interleaved API: (re, im) pairs; split API: real plane */
    void* imag;          /* split API: imaginary plane of a complex array */
    char* str;           /* char arrays; objects: the class name */
    int nfields;         /* struct (1 x 1) / object: named fields / properties */
    char** fnames;
    struct mxArray_tag** fvals;
} mxArray;

int mxGetString(const mxArray* a, char* buf, mwSize len);
double mxGetScalar(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
#if MX_HAS_INTERLEAVED_COMPLEX
double* mxGetDoubles(const mxArray* a);
mxComplexDouble* mxGetComplexDoubles(const mxArray* a);
int64_t* mxGetInt64s(const mxArray* a);
int mxMakeArrayComplex(mxArray* a);
#else
double* mxGetPr(const mxArray* a);
double* mxGetPi(const mxArray* a);
void* mxGetData(const mxArray* a);
#endif
mxLogical* mxGetLogicals(const mxArray* a);
bool mxIsComplex(const mxArray* a);
bool mxIsDouble(const mxArray* a);
bool mxIsNumeric(const mxArray* a);
bool mxIsLogical(const mxArray* a);
bool mxIsChar(const mxArray* a);
mxArray* mxDuplicateArray(const mxArray* a);
void mxDestroyArray(mxArray* a);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity c);
void* mxMalloc(size_t n);
void mxFree(void* p);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...);
/* structs and classdef objects (scalar): mxGetProperty returns a copy the
   caller destroys, mxGetField the struct's own field */
bool mxIsStruct(const mxArray* a);
bool mxIsClass(const mxArray* a, const char* name);
mxArray* mxGetProperty(const mxArray* a, mwSize index, const char* name);
mxArray* mxGetField(const mxArray* a, mwSize index, const char* name);
int mexAtExit(void (*fn)(void));
void mexLock(void);
void mexUnlock(void);

/* test helpers (driver.c / mex_stub.c): element k of a complex array, either API */
void tst_get_c(const mxArray* a, size_t k, double* re, double* im);
void tst_set_c(mxArray* a, size_t k, double re, double im);
/* a scalar struct / object with n named fields (the values are owned by it) */
mxArray* tst_struct(int n, const char* const* names, mxArray** values);
mxArray* tst_object(const char* cls, int n, const char* const* names, mxArray** values);
#endif
