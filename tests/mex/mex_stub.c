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
        case mxDOUBLE_CLASS: return a->cplx && MX_HAS_INTERLEAVED_COMPLEX ? 16 : 8;
        case mxINT64_CLASS: return 8;
        case mxLOGICAL_CLASS: return 1;
        default: return 1;
    }
}
static mxArray* mk(mxClassID c, int cplx, size_t m, size_t n) {
    mxArray* a = calloc(1, sizeof *a);
    a->cls = c; a->cplx = cplx; a->m = m; a->n = n;
    a->data = calloc(m * n != 0 ? m * n : 1, elsize(a));
    if (!MX_HAS_INTERLEAVED_COMPLEX && c == mxDOUBLE_CLASS && cplx) a->imag = calloc(m * n != 0 ? m * n : 1, 8);
    return a;
}
void tst_get_c(const mxArray* a, size_t k, double* re, double* im) {
    if (MX_HAS_INTERLEAVED_COMPLEX) {
        *re = ((double*)a->data)[(a->cplx ? 2 : 1) * k];
        *im = a->cplx ? ((double*)a->data)[2 * k + 1] : 0.0;
    } else {
        *re = ((double*)a->data)[k];
        *im = a->cplx ? ((double*)a->imag)[k] : 0.0;
    }
}
void tst_set_c(mxArray* a, size_t k, double re, double im) {
    if (MX_HAS_INTERLEAVED_COMPLEX) {
        ((double*)a->data)[(a->cplx ? 2 : 1) * k] = re;
        if (a->cplx) ((double*)a->data)[2 * k + 1] = im;
    } else {
        ((double*)a->data)[k] = re;
        if (a->cplx) ((double*)a->imag)[k] = im;
    }
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
#if MX_HAS_INTERLEAVED_COMPLEX
double* mxGetDoubles(const mxArray* a) { return (a->cls == mxDOUBLE_CLASS && !a->cplx) ? a->data : NULL; }
mxComplexDouble* mxGetComplexDoubles(const mxArray* a) { return (a->cls == mxDOUBLE_CLASS && a->cplx) ? a->data : NULL; }
int64_t* mxGetInt64s(const mxArray* a) { return a->cls == mxINT64_CLASS ? a->data : NULL; }
#else
double* mxGetPr(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? a->data : NULL; }
double* mxGetPi(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? a->imag : NULL; }
void* mxGetData(const mxArray* a) { return a->data; }
#endif
mxLogical* mxGetLogicals(const mxArray* a) { return a->cls == mxLOGICAL_CLASS ? a->data : NULL; }
bool mxIsComplex(const mxArray* a) { return a->cplx; }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
bool mxIsNumeric(const mxArray* a) { return a->cls == mxDOUBLE_CLASS || a->cls == mxINT64_CLASS; }
bool mxIsLogical(const mxArray* a) { return a->cls == mxLOGICAL_CLASS; }
bool mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
mxArray* mxDuplicateArray(const mxArray* a) {
    mxArray* b = mk(a->cls, a->cplx, a->m, a->n);
    /* char arrays keep their text in str (driver.c S()), data is a 1-byte dummy */
    if (a->cls != mxCHAR_CLASS) memcpy(b->data, a->data, a->m * a->n * elsize(a));
    if (a->imag) memcpy(b->imag, a->imag, a->m * a->n * 8);
    if (a->str) b->str = strdup(a->str);
    if (a->nfields) {
        b->nfields = a->nfields;
        b->fnames = calloc(a->nfields, sizeof(char*));
        b->fvals = calloc(a->nfields, sizeof(mxArray*));
        for (int i = 0; i < a->nfields; ++i) {
            b->fnames[i] = strdup(a->fnames[i]);
            b->fvals[i] = mxDuplicateArray(a->fvals[i]);
        }
    }
    return b;
}
#if MX_HAS_INTERLEAVED_COMPLEX
int mxMakeArrayComplex(mxArray* a) {
    if (a->cls != mxDOUBLE_CLASS || a->cplx) return a->cplx;
    double* re = a->data;
    double* c = calloc(a->m * a->n != 0 ? 2 * a->m * a->n : 2, 8);
    for (size_t i = 0; i < a->m * a->n; ++i) c[2 * i] = re[i];
    free(re);
    a->data = c;
    a->cplx = 1;
    return 1;
}
#endif
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    for (int i = 0; i < a->nfields; ++i) {
        free(a->fnames[i]);
        mxDestroyArray(a->fvals[i]);
    }
    free(a->fnames);
    free(a->fvals);
    free(a->data); free(a->imag); free(a->str); free(a);
}
mxArray* tst_struct(int n, const char* const* names, mxArray** values) {
    mxArray* a = mk(mxSTRUCT_CLASS, 0, 1, 1);
    a->nfields = n;
    a->fnames = calloc(n ? n : 1, sizeof(char*));
    a->fvals = calloc(n ? n : 1, sizeof(mxArray*));
    for (int i = 0; i < n; ++i) {
        a->fnames[i] = strdup(names[i]);
        a->fvals[i] = values[i];
    }
    return a;
}
mxArray* tst_object(const char* cls, int n, const char* const* names, mxArray** values) {
    mxArray* a = tst_struct(n, names, values);
    a->cls = mxOBJECT_CLASS;
    a->str = strdup(cls);
    return a;
}
bool mxIsStruct(const mxArray* a) { return a->cls == mxSTRUCT_CLASS; }
bool mxIsClass(const mxArray* a, const char* name) { return a->cls == mxOBJECT_CLASS && !strcmp(a->str, name); }
static mxArray* find_field(const mxArray* a, const char* name) {
    for (int i = 0; i < a->nfields; ++i)
        if (!strcmp(a->fnames[i], name)) return a->fvals[i];
    return NULL;
}
mxArray* mxGetField(const mxArray* a, mwSize index, const char* name) {
    return (a->cls == mxSTRUCT_CLASS && index == 0) ? find_field(a, name) : NULL;
}
mxArray* mxGetProperty(const mxArray* a, mwSize index, const char* name) {
    mxArray* v = (a->cls == mxOBJECT_CLASS && index == 0) ? find_field(a, name) : NULL;
    return v ? mxDuplicateArray(v) : NULL;
}
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
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    char msg[256];
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    printf("  warning %s: %s\n", id, msg);
}
int mexAtExit(void (*fn)(void)) { (void)fn; return 0; }
void mexLock(void) {}
void mexUnlock(void) {}

/* ---- recording stub of the C-ABI ----------------------------------------------- */
/* dims of the stub engine: N 540, Ltap 2, LK 336, NP 16, ND 320, 1 scheme, 7 SNR, 4 iter */
enum { SN = 540, STAPS = 2, SLK = 336, SNP = 16, SND = 320, SSNR = 7, SIT = 4 };
struct dsce_ctx { int dummy; };
static struct dsce_ctx g_stub;
static int32_t g_devs[64], g_ndev = 1, g_reduce = 0;
int dsce_create(int dev, dsce_ctx** out) { g_devs[0] = dev; g_ndev = 1; g_reduce = 0; *out = &g_stub; return 0; }
int dsce_create_multi(const int32_t* devs, int32_t n, dsce_ctx** out) {
    int distinct = 1;
    if (n < 1 || n > 64) return DSCE_EINVAL;
    for (int i = 0; i < n; ++i) {
        g_devs[i] = devs[i];                        /* read every entry (ASAN: an undersized list overflows) */
        for (int j = 0; j < i; ++j) distinct = distinct && devs[j] != devs[i];
    }
    g_ndev = n;
    g_reduce = distinct ? 1 : 2;
    printf("  create_multi n=%d reduce=%d\n", n, g_reduce);
    *out = &g_stub;
    return 0;
}
int dsce_group_info(dsce_ctx* c, int32_t* n, int32_t* devs, int32_t* reduce) {
    (void)c;
    if (n) *n = g_ndev;
    if (devs)
        for (int i = 0; i < g_ndev; ++i) devs[i] = g_devs[i];
    if (reduce) *reduce = g_reduce;
    return 0;
}
int dsce_destroy(dsce_ctx* c) { (void)c; return 0; }
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
/* the driver's test arrays (driver.c M()): element i = (1 + i % 7) - (1 + i % 5) j
 * (complex) or 1 + i % 7 (real); the ABI must see them interleaved */
static int interleaved_ok(const double* z, size_t n, int was_complex) {
    for (size_t i = 0; i < n; ++i)
        if (z[2 * i] != 1.0 + (double)(i % 7) || z[2 * i + 1] != (was_complex ? -(1.0 + (double)(i % 5)) : 0.0))
            return 0;
    return 1;
}
int dsce_add_scheme(dsce_ctx* c, const dsce_scheme_desc* d, int32_t* id) {
    (void)c;
    {
        const size_t ng = (size_t)SN * d->n_subcarriers * d->n_symbols;
        const size_t np = (size_t)d->n_subcarriers * d->n_symbols * d->n_tx_symbols;
        printf("  check add_scheme values %s\n",
               interleaved_ok(d->G, ng, 1) && interleaved_ok(d->Q, ng, 1) && interleaved_ok(d->P, np, 0) &&
                       interleaved_ok(d->symbols, (size_t)d->mod_order, 1)
                   ? "OK" : "BAD");
    }
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
    for (int i = 0; i < 2 * SN * STAPS; ++i) ir[i] = i;      /* element k = 2k + (2k + 1) j */
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
    printf("  check mmse_onetap values %s\n", interleaved_ok(hp, (size_t)SNP * n, 1) || interleaved_ok(hp, (size_t)SNP * n, 0) ? "OK" : "BAD");
    for (int i = 0; i < 2 * SLK * n; ++i) h[i] = (i & 1) ? -0.5 * i : a + i;
    return 0;
}
int dsce_set_noise_slot(dsce_ctx* c, int32_t id, int32_t s) { (void)c; (void)id; (void)s; return 0; }
int dsce_set_interpolation(dsce_ctx* c, int32_t id, const double* I) {
    (void)c; (void)id;
    double a = 0.0;
    for (int i = 0; i < 2 * SLK * SNP; ++i) a += I[i];
    printf("  check set_interpolation values %s\n", interleaved_ok(I, (size_t)SLK * SNP, 0) ? "OK" : "BAD");
    printf("  set_interpolation (%g)\n", a != a ? 1.0 : 0.0);
    return 0;
}
int dsce_path_info(dsce_ctx* c, int32_t id, uint32_t* f) { (void)c; (void)id; *f = 0x0f; return 0; }
int dsce_set_option(dsce_ctx* c, const char* n, int64_t v) { (void)c; printf("  set_option %s=%lld\n", n, (long long)v); return 0; }

/* tx_matrices: the descriptor must carry the object's fields as the driver set
   them (driver.c ofdm_object / fbmc_object); G / Q written in full (N x LK) */
int dsce_tx_matrices(dsce_ctx* c, const dsce_tx_desc* d, double* G, double* Q) {
    (void)c;
    const size_t n = (size_t)d->n_samples * d->n_subcarriers * d->n_symbols;
    int ok;
    if (d->kind == 0)
        ok = d->n_subcarriers == 24 && d->n_symbols == 14 && d->n_samples == 540 && d->fft_size == 24 &&
             d->time_spacing == 26 && d->cyclic_prefix == 2 && d->zero_guard == 88 && d->prototype == NULL &&
             d->norm == 1.0 && d->rx_scale == 24.0 * 15e3 / 360e3;
    else
        ok = d->n_subcarriers == 24 && d->n_symbols == 30 && d->n_samples == 540 && d->fft_size == 24 &&
             d->time_spacing == 12 && d->proto_len == 192 && d->prototype && d->prototype[191] == 1.0 + 191 % 7 &&
             d->initial_phase == 0.0 && d->rx_scale == 24.0 / (360e3 * (12.0 / 360e3));
    printf("  check tx_matrices desc %s\n", ok ? "OK" : "BAD");
    for (size_t i = 0; i < 2 * n; ++i) G[i] = (double)i;      /* element k = 2k + (2k+1) j */
    if (Q)
        for (size_t i = 0; i < 2 * n; ++i) Q[i] = (double)i;
    return 0;
}
int dsce_enable_mse(dsce_ctx* c, int32_t on) { (void)c; printf("  enable_mse %d\n", on); return 0; }
int dsce_get_mse(dsce_ctx* c, double* err, double* pw) {
    (void)c;
    for (int i = 0; i < SSNR * (SIT + 1); ++i) err[i] = 0.5 * i;
    for (int i = 0; i < SSNR; ++i) pw[i] = 1.0 + i;
    return 0;
}
int dsce_structured_check(dsce_ctx* c, int32_t id, double* out) {
    (void)c;
    if (id != 0) return DSCE_EINVAL;
    out[0] = 0.07; out[1] = 3e-13; out[2] = 0.59; out[3] = 1e-11; out[4] = 2e-16; out[5] = 1.0; out[6] = 0.01;
    return 0;
}
