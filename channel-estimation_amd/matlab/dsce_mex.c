/*
 * dsce_mex.c — MEX gateway binding the reference's MATLAB host to libdsce.so
 * (include/dsce.h).  Build:
 *   MATLAB R2018a+ (interleaved complex):   mex -R2018a -I../../include dsce_mex.c -L../dsce -ldsce
 *   MATLAB R2013b / R2016a (README.md:19-20, separate real / imaginary planes):
 *                                           mex -I../../include dsce_mex.c -L../dsce -ldsce
 * The complex storage is chosen at compile time by MATLAB's own
 * MX_HAS_INTERLEAVED_COMPLEX (set by -R2018a): with split planes every complex
 * input is interleaved into a scratch array before the ABI call and every
 * complex output is written interleaved to scratch and split into
 * mxGetPr / mxGetPi afterwards (the ABI is interleaved only).
 * MATLAB's mex.h is not part of this image; the gateway's
 * argument checking is exercised on the CPU by tests/test_mex_gateway.py
 * against a test-only mex.h stand-in and a recording stub of the C-ABI.
 *
 * One static context per MATLAB session.  Every command checks its argument
 * count and classes; every output is sized from the engine's own state
 * (dsce_scheme_dims), never from caller arguments.  MATLAB indices (scheme id,
 * SNR index, pilot / data positions) are 1-based here, 0-based at the ABI.
 *
 *   dsce_mex('create' [, device])                                  % device: HIP device (default 0), or a
 *            vector of devices: one multi-device context (dsce_create_multi, ABI 7) whose 'run'
 *            shards the realisations over the devices and sums the counters with one RCCL
 *            all-reduce; every other command is unchanged
 *   [devices, reduce] = dsce_mex('group_info')                      % the context's HIP devices; reduce 0 single
 *            device, 1 RCCL all-reduce, 2 host sum (a device repeats)
 *   dsce_mex('destroy')
 *   dsce_mex('set_channel', SamplingRate, PDPnormalized, N, fD, Paths, DopplerModel)
 *            DopplerModel: 0 'Jakes', 1 'Uniform', 2 'Discrete-Jakes', 3 'Discrete-Uniform'
 *   dsce_mex('set_snr', Pn_time, NrIterations)
 *   id = dsce_mex('add_scheme', L, K, G, Q, P, pilotIdx, dataIdx, considered, symbols,
 *                 kappa, dataDiv, despread, realDetect, bitsSlot, pilotSlot)
 *            G, Q: N x L*K; P: L*K x (NP+ND); pilotIdx: NP; dataIdx: ND (or [] with despread);
 *            considered: ND logical; symbols: M (SymbolMapping sorted by bit label)
 *   dsce_mex('build_mmse' [, ZeroThreshold])                      % default 1e-8
 *   dsce_mex('set_batch', RepsPerBatch)
 *   counts = dsce_mex('run', seed, firstRep, nRep)                % int64 [iter+1, snr, edge, csi, scheme]
 *   bits   = dsce_mex('bits_per_rep', id)                         % [all; no-edge] per realisation
 *   IR     = dsce_mex('channel_realise', seed, rep)               % N x Ltap complex (ImpulseResponse)
 *   W      = dsce_mex('get_W', id, snrIndex, variant)             % (LK^2 NP) x 1 complex; variant 0 W, 1 W0
 *   h      = dsce_mex('mmse_onetap', id, snrIndex, variant, hP)   % LK x n complex, hP: NP x n ('MMSE' slot)
 *   dsce_mex('set_noise_slot', id, slot)
 *   dsce_mex('set_interpolation', id, I)                          % I: LK x NP
 *   d      = dsce_mex('scheme_dims', id)                          % [N Ltap LK NP ND Nsym nSchemes nSNR nIter]
 *   f      = dsce_mex('path_info', id)                            % DSCE_PATH_* bits of the last run
 *   dsce_mex('set_option', name, value)
 *   [G, Q] = dsce_mex('tx_matrices', ModObj)                       % ModObj: Modulation.OFDM or Modulation.FBMC
 *            ('Hermite-OQAM'): G = ModObj.GetTXMatrix, Q = ModObj.GetRXMatrix' (script:191-195) computed
 *            on the GPU from the object's Nr / PHY / Implementation / PrototypeFilter properties
 *   dsce_mex('enable_mse', on)                                      % start (and reset) the MSE sums of 'run'
 *   [err, pow] = dsce_mex('get_mse')                                % err [iter+1, snr, scheme], pow [snr, scheme]
 *   c = dsce_mex('structured_check', id)                           % [ratio, max dev, max |W|, rtol, lr fit, lr eligible, lr ratio]
 */
#ifdef MATLAB_MEX_FILE
#include <math.h>
#include <string.h>

#include "dsce.h"
#include "mex.h"

#ifndef MX_HAS_INTERLEAVED_COMPLEX
#define MX_HAS_INTERLEAVED_COMPLEX 0
#endif

/* real doubles / int64 of an array in either storage API */
#if MX_HAS_INTERLEAVED_COMPLEX
#define DSCE_DOUBLES(a) mxGetDoubles(a)
#define DSCE_INT64S(a) mxGetInt64s(a)
#else
#define DSCE_DOUBLES(a) mxGetPr(a)
#define DSCE_INT64S(a) ((int64_t*)mxGetData(a))
#endif

static dsce_ctx* g_ctx = NULL;

/* teardown status (ABI 6): reported as a warning, since cleanup also runs
 * from mexAtExit where an error cannot be raised */
static void cleanup(void) {
    if (g_ctx && dsce_destroy(g_ctx) != 0)
        mexWarnMsgIdAndTxt("dsce:teardown", "dsce_destroy: a HIP call of the teardown failed (see stderr)");
    g_ctx = NULL;
}

static void check(int rc, const char* what) {
    if (rc != 0) mexErrMsgIdAndTxt("dsce:abi", "%s failed (%d): %s", what, rc, dsce_last_error(g_ctx));
}

/* ---- argument checking ---------------------------------------------------- */
static const char* g_cmd = "";

static void bad(int i, const char* what) {
    mexErrMsgIdAndTxt("dsce:args", "dsce_mex('%s'): argument %d must be %s", g_cmd, i + 1, what);
}

static double scalar(const mxArray* a, int i) {
    if (!mxIsNumeric(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != 1) bad(i, "a real numeric scalar");
    return mxGetScalar(a);
}

static int64_t integer(const mxArray* a, int i, int64_t lo) {
    const double v = scalar(a, i);
    if (v != floor(v) || v < (double)lo || v > 9.007199254740992e15) bad(i, "an integer in range");
    return (int64_t)v;
}

static const double* real_doubles(const mxArray* a, int i, size_t n_expected) {
    if (!mxIsDouble(a) || mxIsComplex(a)) bad(i, "a real double array");
    if (n_expected != (size_t)-1 && mxGetNumberOfElements(a) != n_expected) bad(i, "of the expected length");
    return DSCE_DOUBLES(a);
}

/* interleaved complex view of a double array (the ABI's storage): real inputs
 * are promoted, and with split planes (pre-R2018a) the planes are interleaved,
 * into *tmp (a scratch array the caller destroys) */
static const double* cplx(const mxArray* a, int i, size_t rows, size_t cols, mxArray** tmp) {
    if (!mxIsDouble(a)) bad(i, "a double array");
    if ((rows != (size_t)-1 && mxGetM(a) != rows) || (cols != (size_t)-1 && mxGetN(a) != cols))
        bad(i, "of the expected size");
#if MX_HAS_INTERLEAVED_COMPLEX
    if (mxIsComplex(a)) return (const double*)mxGetComplexDoubles(a);
    *tmp = mxDuplicateArray(a);
    if (!mxMakeArrayComplex(*tmp)) mexErrMsgIdAndTxt("dsce:type", "cannot make argument %d complex", i + 1);
    return (const double*)mxGetComplexDoubles(*tmp);
#else
    {
        const size_t n = mxGetNumberOfElements(a);
        const double* re = mxGetPr(a);
        const double* im = mxIsComplex(a) ? mxGetPi(a) : NULL;
        double* z;
        size_t k;
        *tmp = mxCreateDoubleMatrix((mwSize)(2 * (n ? n : 1)), 1, mxREAL);
        z = mxGetPr(*tmp);
        for (k = 0; k < n; ++k) {
            z[2 * k] = re[k];
            z[2 * k + 1] = im ? im[k] : 0.0;
        }
        return z;
    }
#endif
}

/* A complex output: the ABI writes interleaved (re, im) pairs into the buffer
 * out_begin returns; out_end moves them into the array's storage (split planes
 * before R2018a; nothing to do with interleaved storage). */
typedef struct {
    mxArray* arr;
    mxArray* scratch;
} cplx_out;

static double* out_begin(cplx_out* o, mxArray* arr) {
    o->arr = arr;
    o->scratch = NULL;
#if MX_HAS_INTERLEAVED_COMPLEX
    return (double*)mxGetComplexDoubles(arr);
#else
    {
        const size_t n = mxGetNumberOfElements(arr);
        o->scratch = mxCreateDoubleMatrix((mwSize)(2 * (n ? n : 1)), 1, mxREAL);
        return mxGetPr(o->scratch);
    }
#endif
}

static void out_end(cplx_out* o) {
#if !MX_HAS_INTERLEAVED_COMPLEX
    const size_t n = mxGetNumberOfElements(o->arr);
    const double* z = mxGetPr(o->scratch);
    double *re = mxGetPr(o->arr), *im = mxGetPi(o->arr);
    size_t k;
    for (k = 0; k < n; ++k) {
        re[k] = z[2 * k];
        im[k] = z[2 * k + 1];
    }
#endif
    if (o->scratch) mxDestroyArray(o->scratch);
    o->scratch = NULL;
}

static dsce_dims dims_of(int32_t id) {
    dsce_dims d;
    check(dsce_scheme_dims(g_ctx, id, &d), "dsce_scheme_dims");
    return d;
}

static int32_t scheme_id(const mxArray* a, int i) { return (int32_t)(integer(a, i, 1) - 1); }

/* ---- commands --------------------------------------------------------------- */
typedef void (*cmd_fn)(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

static void c_destroy(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs; (void)plhs; (void)nrhs; (void)prhs;
    cleanup();
    mexUnlock();
}

static void c_set_channel(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    dsce_channel_desc d;
    (void)nlhs; (void)plhs; (void)nrhs;
    d.sampling_rate = scalar(prhs[1], 1);
    d.pdp_norm = real_doubles(prhs[2], 2, (size_t)-1);
    d.n_taps = (int32_t)mxGetNumberOfElements(prhs[2]);
    d.n_samples = (int32_t)integer(prhs[3], 3, 2);
    d.max_doppler = scalar(prhs[4], 4);
    d.n_paths = (int32_t)integer(prhs[5], 5, 1);
    d.doppler_model = (int32_t)integer(prhs[6], 6, 0);
    check(dsce_set_channel(g_ctx, &d), "dsce_set_channel");
}

static void c_set_snr(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs; (void)plhs; (void)nrhs;
    check(dsce_set_snr(g_ctx, real_doubles(prhs[1], 1, (size_t)-1), (int32_t)mxGetNumberOfElements(prhs[1]),
                       (int32_t)integer(prhs[2], 2, 0)), "dsce_set_snr");
}

static void c_add_scheme(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    mxArray *t[4] = {NULL, NULL, NULL, NULL};
    dsce_scheme_desc d;
    size_t np, nd, i, lk, n;
    int32_t *pil, *dat, id;
    uint8_t* cons;
    const double *pp, *dp;
    (void)nlhs; (void)nrhs;
    memset(&d, 0, sizeof d);
    d.n_subcarriers = (int32_t)integer(prhs[1], 1, 1);
    d.n_symbols = (int32_t)integer(prhs[2], 2, 1);
    lk = (size_t)d.n_subcarriers * (size_t)d.n_symbols;
    n = mxGetM(prhs[3]);
    np = mxGetNumberOfElements(prhs[6]);
    nd = mxGetNumberOfElements(prhs[8]);
    d.despread = (int32_t)integer(prhs[12], 12, 0);
    if (!mxIsLogical(prhs[8]) && !mxIsDouble(prhs[8])) bad(8, "a logical or double vector");
    if (mxGetNumberOfElements(prhs[7]) != (d.despread ? mxGetNumberOfElements(prhs[7]) : nd))
        bad(7, "a vector of ND data positions (or [] with despread)");
    d.G = cplx(prhs[3], 3, n, lk, &t[0]);
    d.Q = cplx(prhs[4], 4, n, lk, &t[1]);
    d.P = cplx(prhs[5], 5, lk, np + nd, &t[2]);
    pp = real_doubles(prhs[6], 6, np);
    dp = mxGetNumberOfElements(prhs[7]) ? real_doubles(prhs[7], 7, nd) : NULL;
    d.symbols = cplx(prhs[9], 9, (size_t)-1, (size_t)-1, &t[3]);
    pil = mxMalloc((np ? np : 1) * sizeof(int32_t));
    dat = mxMalloc((nd ? nd : 1) * sizeof(int32_t));
    cons = mxMalloc(nd ? nd : 1);
    for (i = 0; i < np; ++i) pil[i] = (int32_t)pp[i] - 1;
    for (i = 0; i < nd; ++i) {
        dat[i] = dp ? (int32_t)dp[i] - 1 : 0;
        cons[i] = mxIsLogical(prhs[8]) ? (mxGetLogicals(prhs[8])[i] ? 1 : 0) : (DSCE_DOUBLES(prhs[8])[i] != 0.0);
    }
    d.n_tx_symbols = (int32_t)(np + nd);
    d.n_pilots = (int32_t)np;
    d.n_data = (int32_t)nd;
    d.pilot_pos = pil;
    d.data_pos = dat;
    d.considered = cons;
    d.mod_order = (int32_t)mxGetNumberOfElements(prhs[9]);
    for (d.bits_per_symbol = 0; (1 << d.bits_per_symbol) < d.mod_order && d.bits_per_symbol < 30; ++d.bits_per_symbol) {}
    d.kappa = scalar(prhs[10], 10);
    d.data_div = scalar(prhs[11], 11);
    d.real_detect = (int32_t)integer(prhs[13], 13, 0);
    d.bits_slot = (int32_t)integer(prhs[14], 14, 0);
    d.pilot_slot = (int32_t)integer(prhs[15], 15, 0);
    {
        const int rc = dsce_add_scheme(g_ctx, &d, &id);
        mxFree(pil);
        mxFree(dat);
        mxFree(cons);
        for (i = 0; i < 4; ++i)
            if (t[i]) mxDestroyArray(t[i]);
        check(rc, "dsce_add_scheme");
    }
    plhs[0] = mxCreateDoubleScalar(id + 1);
}

static void c_build_mmse(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs; (void)plhs;
    check(dsce_build_mmse(g_ctx, nrhs > 1 ? scalar(prhs[1], 1) : 1e-8), "dsce_build_mmse");
}

static void c_set_batch(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs; (void)plhs; (void)nrhs;
    check(dsce_set_batch(g_ctx, (int32_t)integer(prhs[1], 1, 64)), "dsce_set_batch");
}

static void c_run(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* counts are C-ordered [scheme][csi][edge][snr][stage]: reversed dims in MATLAB */
    const dsce_dims d = dims_of(0);
    mwSize dm[5];
    (void)nlhs; (void)nrhs;
    dm[0] = (mwSize)(d.n_iter + 1); dm[1] = (mwSize)d.n_snr; dm[2] = 2; dm[3] = 2; dm[4] = (mwSize)d.n_schemes;
    plhs[0] = mxCreateNumericArray(5, dm, mxINT64_CLASS, mxREAL);
    if ((int64_t)mxGetNumberOfElements(plhs[0]) != d.n_counters) mexErrMsgIdAndTxt("dsce:state", "counter shape");
    /* any nRep >= 0: the script's NrRepetitions (script:19 / :44) as is */
    check(dsce_run(g_ctx, (uint64_t)integer(prhs[1], 1, 0), (uint64_t)integer(prhs[2], 2, 0),
                   (uint64_t)integer(prhs[3], 3, 0), DSCE_INT64S(plhs[0])), "dsce_run");
}

static void c_bits_per_rep(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    int64_t b[2];
    (void)nlhs; (void)nrhs;
    check(dsce_bits_per_rep(g_ctx, scheme_id(prhs[1], 1), b), "dsce_bits_per_rep");
    plhs[0] = mxCreateDoubleMatrix(2, 1, mxREAL);
    DSCE_DOUBLES(plhs[0])[0] = (double)b[0];
    DSCE_DOUBLES(plhs[0])[1] = (double)b[1];
}

static void c_channel_realise(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    const dsce_dims d = dims_of(0);
    (void)nlhs; (void)nrhs;
    cplx_out o;
    double* z;
    int rc;
    plhs[0] = mxCreateDoubleMatrix((mwSize)d.n_samples, (mwSize)d.n_taps, mxCOMPLEX);
    z = out_begin(&o, plhs[0]);
    rc = dsce_channel_realise(g_ctx, (uint64_t)integer(prhs[1], 1, 0), (uint64_t)integer(prhs[2], 2, 0), z);
    out_end(&o);
    check(rc, "dsce_channel_realise");
}

static void c_get_W(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    const int32_t id = scheme_id(prhs[1], 1);
    const dsce_dims d = dims_of(id);
    (void)nlhs; (void)nrhs;
    const int32_t k = (int32_t)integer(prhs[2], 2, 1) - 1, var = (int32_t)integer(prhs[3], 3, 0);
    cplx_out o;
    double* z;
    int rc;
    plhs[0] = mxCreateDoubleMatrix((mwSize)d.lk * (mwSize)d.lk * (mwSize)d.n_pilots, 1, mxCOMPLEX);
    z = out_begin(&o, plhs[0]);
    rc = dsce_get_W(g_ctx, id, k, var, z);
    out_end(&o);
    check(rc, "dsce_get_W");
}

static void c_mmse_onetap(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* the 'MMSE' slot of PilotSymbolAidedChannelEstimation (PSACE.m:128-129) */
    const int32_t id = scheme_id(prhs[1], 1);
    const dsce_dims d = dims_of(id);
    mxArray* t = NULL;
    const double* hp;
    size_t n;
    int32_t k, var;
    cplx_out o;
    double* z;
    (void)nlhs; (void)nrhs;
    if (mxGetM(prhs[4]) != (size_t)d.n_pilots) bad(4, "an NP x n matrix of LS pilot estimates");
    n = mxGetN(prhs[4]);
    if (n < 1) bad(4, "non-empty");
    k = (int32_t)integer(prhs[2], 2, 1) - 1;
    var = (int32_t)integer(prhs[3], 3, 0);
    hp = cplx(prhs[4], 4, (size_t)d.n_pilots, n, &t);
    plhs[0] = mxCreateDoubleMatrix((mwSize)d.lk, (mwSize)n, mxCOMPLEX);
    z = out_begin(&o, plhs[0]);
    {
        const int rc = dsce_mmse_onetap(g_ctx, id, k, var, hp, (int32_t)n, z);
        out_end(&o);
        if (t) mxDestroyArray(t);
        check(rc, "dsce_mmse_onetap");
    }
}

static void c_set_noise_slot(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* SimpleVersion_DoublyFlat.m:125-126 */
    (void)nlhs; (void)plhs; (void)nrhs;
    check(dsce_set_noise_slot(g_ctx, scheme_id(prhs[1], 1), (int32_t)integer(prhs[2], 2, 0)), "dsce_set_noise_slot");
}

static void c_set_interpolation(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* I = LK x NP weights of a PilotSymbolAidedChannelEstimation ('linear',
       'MovingBlockAverage', ...), e.g. ChannelInterpolation of the NP unit vectors */
    const int32_t id = scheme_id(prhs[1], 1);
    const dsce_dims d = dims_of(id);
    mxArray* t = NULL;
    const double* I;
    (void)nlhs; (void)plhs; (void)nrhs;
    I = cplx(prhs[2], 2, (size_t)d.lk, (size_t)d.n_pilots, &t);
    {
        const int rc = dsce_set_interpolation(g_ctx, id, I);
        if (t) mxDestroyArray(t);
        check(rc, "dsce_set_interpolation");
    }
}

static void c_scheme_dims(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    const dsce_dims d = dims_of(scheme_id(prhs[1], 1));
    double* o;
    (void)nlhs; (void)nrhs;
    plhs[0] = mxCreateDoubleMatrix(1, 9, mxREAL);
    o = DSCE_DOUBLES(plhs[0]);
    o[0] = d.n_samples; o[1] = d.n_taps; o[2] = d.lk; o[3] = d.n_pilots; o[4] = d.n_data;
    o[5] = d.n_tx_symbols; o[6] = d.n_schemes; o[7] = d.n_snr; o[8] = d.n_iter;
}

static void c_path_info(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    uint32_t f = 0;
    (void)nlhs; (void)nrhs;
    check(dsce_path_info(g_ctx, scheme_id(prhs[1], 1), &f), "dsce_path_info");
    plhs[0] = mxCreateDoubleScalar((double)f);
}

static void c_set_option(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char name[64];
    (void)nlhs; (void)plhs; (void)nrhs;
    if (!mxIsChar(prhs[1]) || mxGetString(prhs[1], name, sizeof name)) bad(1, "an option name");
    check(dsce_set_option(g_ctx, name, integer(prhs[2], 2, -1)), "dsce_set_option");
}


/* ---- Modulation.OFDM / Modulation.FBMC objects (tx_matrices) ------------------- */
/* property `prop` (a struct) of the object, field `field` as a real scalar */
static const mxArray* g_props[4];                 /* owned copies from mxGetProperty, freed by props_free */
static int g_nprops = 0;
static void props_free(void) {
    int i;
    for (i = 0; i < g_nprops; ++i) mxDestroyArray((mxArray*)g_props[i]);
    g_nprops = 0;
}
static const mxArray* prop(const mxArray* obj, const char* name) {
    mxArray* p = mxGetProperty(obj, 0, name);            /* a copy (MATLAB semantics) */
    if (!p || !mxIsStruct(p)) {
        if (p) mxDestroyArray(p);
        props_free();
        mexErrMsgIdAndTxt("dsce:args", "dsce_mex('tx_matrices'): the object has no struct property %s", name);
    }
    g_props[g_nprops++] = p;
    return p;
}
static double field(const mxArray* st, const char* name) {
    const mxArray* f = mxGetField(st, 0, name);
    if (!f || !mxIsNumeric(f) || mxIsComplex(f) || mxGetNumberOfElements(f) != 1) {
        props_free();
        mexErrMsgIdAndTxt("dsce:args", "dsce_mex('tx_matrices'): field %s must be a real scalar", name);
    }
    return mxGetScalar(f);
}

static void c_tx_matrices(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* OFDM.m:184-218 / FBMC.m:318-354 on the GPU (dsce_tx_matrices, row f1) */
    const mxArray* obj = prhs[1];
    const mxArray *nr, *phy, *im, *pf, *td;
    mxArray* meth;
    dsce_tx_desc d;
    cplx_out og, oq;
    double *zg, *zq;
    size_t lk;
    int fbmc, rc;
    (void)nrhs;
    if (mxIsClass(obj, "Modulation.OFDM")) fbmc = 0;
    else if (mxIsClass(obj, "Modulation.FBMC")) fbmc = 1;
    else bad(1, "a Modulation.OFDM or Modulation.FBMC object");
    memset(&d, 0, sizeof d);
    nr = prop(obj, "Nr");
    phy = prop(obj, "PHY");
    im = prop(obj, "Implementation");
    if (field(phy, "TransmitRealSignal") != 0.0) {
        props_free();
        mexErrMsgIdAndTxt("dsce:args", "dsce_mex('tx_matrices'): PHY.TransmitRealSignal must be false (OFDM.m:188-191)");
    }
    d.kind = fbmc;
    d.n_subcarriers = (int32_t)field(nr, "Subcarriers");
    d.n_symbols = (int32_t)field(nr, "MCSymbols");
    d.n_samples = (int32_t)field(nr, "SamplesTotal");
    d.fft_size = (int32_t)field(im, "FFTSize");
    d.intermediate_bin = (int32_t)field(im, "IntermediateFrequency");
    d.time_spacing = (int32_t)field(im, "TimeSpacing");
    d.norm = field(im, "NormalizationFactor");
    if (fbmc) {
        char m[32];
        meth = mxGetProperty(obj, 0, "Method");
        if (!meth || mxGetString(meth, m, sizeof m) || strcmp(m, "Hermite-OQAM")) {
            if (meth) mxDestroyArray(meth);
            props_free();
            mexErrMsgIdAndTxt("dsce:args", "dsce_mex('tx_matrices'): FBMC Method must be 'Hermite-OQAM'");
        }
        mxDestroyArray(meth);
        pf = prop(obj, "PrototypeFilter");
        td = mxGetField(pf, 0, "TimeDomain");
        if (!td || !mxIsDouble(td) || mxIsComplex(td)) {
            props_free();
            mexErrMsgIdAndTxt("dsce:args", "dsce_mex('tx_matrices'): PrototypeFilter.TimeDomain must be real");
        }
        d.proto_len = (int32_t)mxGetNumberOfElements(td);
        d.prototype = DSCE_DOUBLES(td);
        d.initial_phase = field(im, "InitialPhaseShift");
        d.rx_scale = field(nr, "Subcarriers") / (field(phy, "SamplingRate") * field(phy, "TimeSpacing"));   /* FBMC.m:352 */
    } else {
        d.cyclic_prefix = (int32_t)field(im, "CyclicPrefix");
        d.zero_guard = (int32_t)field(im, "ZeroGuardSamples");
        d.rx_scale = field(nr, "Subcarriers") * field(phy, "SubcarrierSpacing") / field(phy, "SamplingRate");  /* OFDM.m:214 */
    }
    lk = (size_t)d.n_subcarriers * (size_t)d.n_symbols;
    plhs[0] = mxCreateDoubleMatrix((mwSize)d.n_samples, (mwSize)lk, mxCOMPLEX);
    zg = out_begin(&og, plhs[0]);
    zq = NULL;
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix((mwSize)d.n_samples, (mwSize)lk, mxCOMPLEX);
        zq = out_begin(&oq, plhs[1]);
    }
    rc = dsce_tx_matrices(g_ctx, &d, zg, zq);
    out_end(&og);
    if (nlhs > 1) out_end(&oq);
    props_free();
    check(rc, "dsce_tx_matrices");
}

static void c_enable_mse(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs; (void)plhs; (void)nrhs;
    check(dsce_enable_mse(g_ctx, (int32_t)integer(prhs[1], 1, 0)), "dsce_enable_mse");
}

static void c_get_mse(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    /* C-ordered err [scheme][snr][stage], pow [scheme][snr]: reversed dims in MATLAB */
    const dsce_dims d = dims_of(0);
    mwSize de[3];
    mxArray* pw;
    (void)nrhs; (void)prhs;
    de[0] = (mwSize)(d.n_iter + 1); de[1] = (mwSize)d.n_snr; de[2] = (mwSize)d.n_schemes;
    plhs[0] = mxCreateNumericArray(3, de, mxDOUBLE_CLASS, mxREAL);
    pw = mxCreateDoubleMatrix((mwSize)d.n_snr, (mwSize)d.n_schemes, mxREAL);
    {
        const int rc = dsce_get_mse(g_ctx, DSCE_DOUBLES(plhs[0]), DSCE_DOUBLES(pw));
        if (rc != 0) mxDestroyArray(pw);
        check(rc, "dsce_get_mse");
    }
    if (nlhs > 1) plhs[1] = pw;
    else mxDestroyArray(pw);
}

static void c_group_info(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    int32_t n = 0, red = 0, k;
    int32_t devs[64];
    (void)nrhs; (void)prhs;
    check(dsce_group_info(g_ctx, &n, NULL, NULL), "dsce_group_info");
    if (n < 1 || n > 64) mexErrMsgIdAndTxt("dsce:state", "group size");
    check(dsce_group_info(g_ctx, NULL, devs, &red), "dsce_group_info");
    plhs[0] = mxCreateDoubleMatrix(1, (mwSize)n, mxREAL);
    for (k = 0; k < n; ++k) DSCE_DOUBLES(plhs[0])[k] = devs[k];
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(red);
}

static void c_structured_check(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    double c[7];
    int k;
    (void)nlhs; (void)nrhs;
    check(dsce_structured_check(g_ctx, scheme_id(prhs[1], 1), c), "dsce_structured_check");
    plhs[0] = mxCreateDoubleMatrix(1, 7, mxREAL);
    for (k = 0; k < 7; ++k) DSCE_DOUBLES(plhs[0])[k] = c[k];
}

static const struct {
    const char* name;
    int nrhs_min, nrhs_max, nlhs;
    cmd_fn fn;
} CMDS[] = {
    {"destroy", 1, 1, 0, c_destroy},
    {"set_channel", 7, 7, 0, c_set_channel},
    {"set_snr", 3, 3, 0, c_set_snr},
    {"add_scheme", 16, 16, 1, c_add_scheme},
    {"build_mmse", 1, 2, 0, c_build_mmse},
    {"set_batch", 2, 2, 0, c_set_batch},
    {"run", 4, 4, 1, c_run},
    {"bits_per_rep", 2, 2, 1, c_bits_per_rep},
    {"channel_realise", 3, 3, 1, c_channel_realise},
    {"get_W", 4, 4, 1, c_get_W},
    {"mmse_onetap", 5, 5, 1, c_mmse_onetap},
    {"set_noise_slot", 3, 3, 0, c_set_noise_slot},
    {"set_interpolation", 3, 3, 0, c_set_interpolation},
    {"scheme_dims", 2, 2, 1, c_scheme_dims},
    {"path_info", 2, 2, 1, c_path_info},
    {"set_option", 3, 3, 0, c_set_option},
    {"tx_matrices", 2, 2, 2, c_tx_matrices},
    {"enable_mse", 2, 2, 0, c_enable_mse},
    {"get_mse", 1, 1, 2, c_get_mse},
    {"structured_check", 2, 2, 1, c_structured_check},
    {"group_info", 1, 1, 2, c_group_info},
};

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char cmd[32];
    size_t i;
    if (nrhs < 1 || !mxIsChar(prhs[0]) || mxGetString(prhs[0], cmd, sizeof cmd))
        mexErrMsgIdAndTxt("dsce:usage", "dsce_mex(cmd, ...): cmd must be a command name");
    g_cmd = cmd;
    if (!strcmp(cmd, "create")) {
        if (nrhs > 2) mexErrMsgIdAndTxt("dsce:usage", "dsce_mex('create' [, device or device vector])");
        if (nrhs > 1 && mxGetNumberOfElements(prhs[1]) != 1) {
            /* a device vector: one multi-device context (dsce_create_multi) */
            int32_t devs[64];
            const size_t n = mxGetNumberOfElements(prhs[1]);
            const double* d;
            size_t k;
            if (n < 1 || n > 64) bad(1, "a device or a vector of 1 to 64 devices");
            d = real_doubles(prhs[1], 1, n);
            for (k = 0; k < n; ++k) {
                if (d[k] != floor(d[k]) || d[k] < 0 || d[k] > 1e6) bad(1, "a vector of device indices >= 0");
                devs[k] = (int32_t)d[k];
            }
            cleanup();
            check(dsce_create_multi(devs, (int32_t)n, &g_ctx), "dsce_create_multi");
        } else {
            const int dev = nrhs > 1 ? (int)integer(prhs[1], 1, 0) : 0;
            cleanup();
            check(dsce_create(dev, &g_ctx), "dsce_create");
        }
        mexAtExit(cleanup);
        mexLock();
        return;
    }
    for (i = 0; i < sizeof CMDS / sizeof CMDS[0]; ++i) {
        if (strcmp(cmd, CMDS[i].name)) continue;
        if (nrhs < CMDS[i].nrhs_min || nrhs > CMDS[i].nrhs_max)
            mexErrMsgIdAndTxt("dsce:usage", "dsce_mex('%s'): expected %d to %d arguments, got %d", cmd,
                              CMDS[i].nrhs_min, CMDS[i].nrhs_max, nrhs);
        if (nlhs > CMDS[i].nlhs) mexErrMsgIdAndTxt("dsce:usage", "dsce_mex('%s'): too many outputs", cmd);
        if (!g_ctx) mexErrMsgIdAndTxt("dsce:state", "call dsce_mex('create') first");
        CMDS[i].fn(nlhs, plhs, nrhs, prhs);
        return;
    }
    mexErrMsgIdAndTxt("dsce:usage", "unknown command '%s'", cmd);
}
#endif /* MATLAB_MEX_FILE */
