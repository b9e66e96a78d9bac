/* TEST-ONLY: implementation of tests/mex/mex.h and a recording stub of the
 * C-ABI (include/dsce.h) with fixed dimensions.  Every stubbed call writes
 * exactly as many elements as the real engine would, so an output the gateway
 * sized too small is a heap overflow that AddressSanitizer reports. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsce.h"
#include "mex.h"

jmp_buf g_err_jmp;
char g_err_id[64];

/* ---- mex / mx ---------------------------------------------------------- */
static size_t elsize(const mxArray* a) {
    switch (a->cls) {
        case mxDOUBLE_CLASS: return a->cplx ? 16 : 8;
        case mxINT64_CLASS: return 8;
        case mxLOGICAL_CLASS: return 1;
        default: return 1;
    }
}
static mxArray* mk(mxClassID c, int cplx, size_t m, size_t n) {
    mxArray* a = calloc(1, sizeof *a);
    a->cls = c; a->cplx = cplx; a->m = m; a->n = n;
    a->data = calloc(m * n ? m * n : 1, elsize(a));
    return a;
}
int mxGetString(const mxArray* a, char* buf, mwSize len) {
    if (a->cls != mxCHAR_CLASS || strlen(a->str) + 1 > len) return 1;
    strcpy(buf, a->str);
    return 0;
}
double mxGetScalar(const mxArray* a) {
    if (a->cls == mxDOUBLE_CLASS) return ((double*)a->data)[0];
    if (a->cls == mxLOGICAL_CLASS) return ((mxLogical*)a->data)[0];
    if (a->cls == mxINT64_CLASS) return (double)((int64_t*)a->data)[0];
    return 0.0;
}
size_t mxGetNumberOfElements(const mxArray* a) { return a->m * a->n; }
size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
double* mxGetDoubles(const mxArray* a) { return (a->cls == mxDOUBLE_CLASS && !a->cplx) ? a->data : NULL; }
mxComplexDouble* mxGetComplexDoubles(const mxArray* a) { return (a->cls == mxDOUBLE_CLASS && a->cplx) ? a->data : NULL; }
mxLogical* mxGetLogicals(const mxArray* a) { return a->cls == mxLOGICAL_CLASS ? a->data : NULL; }
int64_t* mxGetInt64s(const mxArray* a) { return a->cls == mxINT64_CLASS ? a->data : NULL; }
bool mxIsComplex(const mxArray* a) { return a->cplx; }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
bool mxIsNumeric(const mxArray* a) { return a->cls == mxDOUBLE_CLASS || a->cls == mxINT64_CLASS; }
bool mxIsLogical(const mxArray* a) { return a->cls == mxLOGICAL_CLASS; }
bool mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
mxArray* mxDuplicateArray(const mxArray* a) {
    mxArray* b = mk(a->cls, a->cplx, a->m, a->n);
    memcpy(b->data, a->data, a->m * a->n * elsize(a));
    return b;
}
int mxMakeArrayComplex(mxArray* a) {
    if (a->cls != mxDOUBLE_CLASS || a->cplx) return a->cplx;
    double* re = a->data;
    double* c = calloc(a->m * a->n ? 2 * a->m * a->n : 2, 8);
    for (size_t i = 0; i < a->m * a->n; ++i) c[2 * i] = re[i];
    free(re);
    a->data = c;
    a->cplx = 1;
    return 1;
}
void mxDestroyArray(mxArray* a) { if (a) { free(a->data); free(a->str); free(a); } }
mxArray* mxCreateDoubleScalar(double v) { mxArray* a = mk(mxDOUBLE_CLASS, 0, 1, 1); ((double*)a->data)[0] = v; return a; }
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) { return mk(mxDOUBLE_CLASS, c == mxCOMPLEX, m, n); }
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity c) {
    size_t n = 1;
    for (mwSize i = 1; i < nd; ++i) n *= dims[i];
    return mk(cls, c == mxCOMPLEX, dims[0], n);
}
void* mxMalloc(size_t n) { return malloc(n); }
void mxFree(void* p) { free(p); }
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    char msg[256];
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    snprintf(g_err_id, sizeof g_err_id, "%s", id);
    printf("  error %s: %s\n", id, msg);
    longjmp(g_err_jmp, 1);
}
int mexAtExit(void (*fn)(void)) { (void)fn; return 0; }
void mexLock(void) {}
void mexUnlock(void) {}

/* ---- recording stub of the C-ABI ----------------------------------------------- */
/* dims of the stub engine: N 540, Ltap 2, LK 336, NP 16, ND 320, 1 scheme, 7 SNR, 4 iter */
enum { SN = 540, STAPS = 2, SLK = 336, SNP = 16, SND = 320, SSNR = 7, SIT = 4 };
struct dsce_ctx { int dummy; };
static struct dsce_ctx g_stub;
int dsce_create(int dev, dsce_ctx** out) { (void)dev; *out = &g_stub; return 0; }
void dsce_destroy(dsce_ctx* c) { (void)c; }
const char* dsce_last_error(const dsce_ctx* c) { (void)c; return "stub"; }
int dsce_scheme_dims(dsce_ctx* c, int32_t id, dsce_dims* d) {
    (void)c;
    if (id != 0) return DSCE_EINVAL;
    d->n_samples = SN; d->n_taps = STAPS; d->lk = SLK; d->n_pilots = SNP; d->n_data = SND;
    d->n_tx_symbols = SNP + SND; d->n_schemes = 1; d->n_snr = SSNR; d->n_iter = SIT;
    d->n_counters = 1LL * 4 * SSNR * (SIT + 1);
    return 0;
}
int dsce_set_channel(dsce_ctx* c, const dsce_channel_desc* d) { (void)c; printf("  set_channel N=%d taps=%d\n", d->n_samples, d->n_taps); return 0; }
int dsce_set_snr(dsce_ctx* c, const double* p, int32_t n, int32_t it) { (void)c; (void)p; printf("  set_snr %d %d\n", n, it); return 0; }
int dsce_add_scheme(dsce_ctx* c, const dsce_scheme_desc* d, int32_t* id) {
    (void)c;
    /* read every input like the engine does */
    double acc = 0.0;
    size_t n = (size_t)SN * d->n_subcarriers * d->n_symbols;
    for (size_t i = 0; i < 2 * n; ++i) acc += d->G[i] + d->Q[i];
    for (size_t i = 0; i < 2 * (size_t)d->n_subcarriers * d->n_symbols * d->n_tx_symbols; ++i) acc += d->P[i];
    for (int i = 0; i < d->n_pilots; ++i) acc += d->pilot_pos[i];
    for (int i = 0; i < d->n_data; ++i) acc += d->data_pos[i] + d->considered[i];
    for (int i = 0; i < 2 * d->mod_order; ++i) acc += d->symbols[i];
    printf("  add_scheme L=%d K=%d NP=%d ND=%d M=%d bits=%d pil0=%d (%g)\n", d->n_subcarriers, d->n_symbols,
           d->n_pilots, d->n_data, d->mod_order, d->bits_per_symbol, d->pilot_pos[0], acc != acc ? 1.0 : 0.0);
    *id = 0;
    return 0;
}
int dsce_build_mmse(dsce_ctx* c, double t) { (void)c; printf("  build_mmse %g\n", t); return 0; }
int dsce_set_batch(dsce_ctx* c, int32_t r) { (void)c; printf("  set_batch %d\n", r); return 0; }
int dsce_run(dsce_ctx* c, uint64_t s, uint64_t f, uint64_t n, int64_t* e) {
    (void)c; (void)s; (void)f; (void)n;
    for (int i = 0; i < 4 * SSNR * (SIT + 1); ++i) e[i] += i;
    return 0;
}
int dsce_bits_per_rep(dsce_ctx* c, int32_t id, int64_t* b) { (void)c; (void)id; b[0] = 2560; b[1] = 1280; return 0; }
int dsce_channel_realise(dsce_ctx* c, uint64_t s, uint64_t r, double* ir) {
    (void)c; (void)s; (void)r;
    for (int i = 0; i < 2 * SN * STAPS; ++i) ir[i] = i;
    return 0;
}
int dsce_get_W(dsce_ctx* c, int32_t id, int32_t k, int32_t v, double* w) {
    (void)c; (void)id;
    if (k < 0 || k >= SSNR || v < 0 || v > 1) return DSCE_EINVAL;
    for (size_t i = 0; i < 2ull * SLK * SLK * SNP; ++i) w[i] = 0.5;
    return 0;
}
int dsce_mmse_onetap(dsce_ctx* c, int32_t id, int32_t k, int32_t v, const double* hp, int32_t n, double* h) {
    (void)c; (void)id; (void)v;
    double a = 0.0;
    if (k < 0 || k >= SSNR) return DSCE_EINVAL;
    for (int i = 0; i < 2 * SNP * n; ++i) a += hp[i];
    for (int i = 0; i < 2 * SLK * n; ++i) h[i] = a;
    return 0;
}
int dsce_set_noise_slot(dsce_ctx* c, int32_t id, int32_t s) { (void)c; (void)id; (void)s; return 0; }
int dsce_set_interpolation(dsce_ctx* c, int32_t id, const double* I) {
    (void)c; (void)id;
    double a = 0.0;
    for (int i = 0; i < 2 * SLK * SNP; ++i) a += I[i];
    printf("  set_interpolation (%g)\n", a != a ? 1.0 : 0.0);
    return 0;
}
int dsce_path_info(dsce_ctx* c, int32_t id, uint32_t* f) { (void)c; (void)id; *f = 0x0f; return 0; }
int dsce_set_option(dsce_ctx* c, const char* n, int64_t v) { (void)c; printf("  set_option %s=%lld\n", n, (long long)v); return 0; }
