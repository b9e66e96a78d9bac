/*
 * dsce_mex.c — MEX gateway binding the reference's MATLAB host to libdsce.so.
 * Build (MATLAB R2018a+, interleaved complex):
 *   mex -R2018a -I../../include dsce_mex.c -L../dsce -ldsce
 * Requires MATLAB's mex.h, which is not part of this image.
 *
 * Usage from MATLAB (one static context per MATLAB session, device 0 or set):
 *   dsce_mex('create', device)
 *   dsce_mex('set_channel', SamplingRate, PDPnormalized, N, fD, Paths, isUniform)
 *   dsce_mex('set_snr', Pn_time, NrIterations)
 *   id = dsce_mex('add_scheme', L, K, G, Q, P, pilotIdx, dataIdx, considered, symbols,
 *                 kappa, dataDiv, despread, realDetect, bitsSlot, pilotSlot)
 *   dsce_mex('build_mmse', 1e-8)
 *   counts = dsce_mex('run', seed, firstRep, nRep)        % int64 [iter+1, snr, 2, 2, schemes]
 *   IR = dsce_mex('channel_realise', seed, rep)            % N x Ltap complex
 *   W  = dsce_mex('get_W', id, snrIndex, variant)          % LK^2*NP x 1 complex
 *   dsce_mex('destroy')
 * MATLAB indices (pilotIdx, dataIdx, snrIndex, id) are 1-based here and
 * converted to the ABI's 0-based convention.
 */
#ifdef MATLAB_MEX_FILE
#include <string.h>

#include "dsce.h"
#include "mex.h"

static dsce_ctx* g_ctx = NULL;

static void cleanup(void) {
    if (g_ctx) dsce_destroy(g_ctx);
    g_ctx = NULL;
}

static void check(int rc, const char* what) {
    if (rc != 0) mexErrMsgIdAndTxt("dsce:abi", "%s failed (%d): %s", what, rc, dsce_last_error(g_ctx));
}

static double* cplx(const mxArray* a, mxArray** tmp) {
    /* interleaved complex view; real inputs are promoted */
    if (mxIsComplex(a)) return (double*)mxGetComplexDoubles(a);
    *tmp = mxDuplicateArray(a);
    if (!mxMakeArrayComplex(*tmp)) mexErrMsgIdAndTxt("dsce:type", "cannot make complex");
    return (double*)mxGetComplexDoubles(*tmp);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char cmd[32];
    if (nrhs < 1 || mxGetString(prhs[0], cmd, sizeof cmd)) mexErrMsgIdAndTxt("dsce:usage", "dsce_mex(cmd, ...)");
    if (!strcmp(cmd, "create")) {
        cleanup();
        check(dsce_create(nrhs > 1 ? (int)mxGetScalar(prhs[1]) : 0, &g_ctx), "dsce_create");
        mexAtExit(cleanup);
        mexLock();
        return;
    }
    if (!g_ctx) mexErrMsgIdAndTxt("dsce:state", "call dsce_mex('create') first");
    if (!strcmp(cmd, "destroy")) {
        cleanup();
        mexUnlock();
    } else if (!strcmp(cmd, "set_channel")) {
        dsce_channel_desc d;
        d.sampling_rate = mxGetScalar(prhs[1]);
        d.pdp_norm = mxGetDoubles(prhs[2]);
        d.n_taps = (int32_t)mxGetNumberOfElements(prhs[2]);
        d.n_samples = (int32_t)mxGetScalar(prhs[3]);
        d.max_doppler = mxGetScalar(prhs[4]);
        d.n_paths = (int32_t)mxGetScalar(prhs[5]);
        d.doppler_model = (int32_t)mxGetScalar(prhs[6]);
        check(dsce_set_channel(g_ctx, &d), "dsce_set_channel");
    } else if (!strcmp(cmd, "set_snr")) {
        check(dsce_set_snr(g_ctx, mxGetDoubles(prhs[1]), (int32_t)mxGetNumberOfElements(prhs[1]),
                           (int32_t)mxGetScalar(prhs[2])), "dsce_set_snr");
    } else if (!strcmp(cmd, "add_scheme")) {
        mxArray *t1 = NULL, *t2 = NULL, *t3 = NULL, *t4 = NULL;
        dsce_scheme_desc d;
        size_t np = mxGetNumberOfElements(prhs[6]), nd = mxGetNumberOfElements(prhs[8]), i;
        int32_t *pil = mxMalloc(np * sizeof(int32_t)), *dat = mxMalloc(nd * sizeof(int32_t));
        uint8_t* cons = mxMalloc(nd);
        const double* pp = mxGetDoubles(prhs[6]);
        const double* dp = mxGetNumberOfElements(prhs[7]) ? mxGetDoubles(prhs[7]) : NULL;
        const mxLogical* cp = mxGetLogicals(prhs[8]);
        int32_t id;
        for (i = 0; i < np; ++i) pil[i] = (int32_t)pp[i] - 1;
        for (i = 0; i < nd; ++i) { dat[i] = dp ? (int32_t)dp[i] - 1 : 0; cons[i] = cp[i] ? 1 : 0; }
        d.n_subcarriers = (int32_t)mxGetScalar(prhs[1]);
        d.n_symbols = (int32_t)mxGetScalar(prhs[2]);
        d.G = cplx(prhs[3], &t1);
        d.Q = cplx(prhs[4], &t2);
        d.P = cplx(prhs[5], &t3);
        d.n_tx_symbols = (int32_t)mxGetN(prhs[5]);
        d.n_pilots = (int32_t)np;
        d.n_data = (int32_t)nd;
        d.pilot_pos = pil;
        d.data_pos = dat;
        d.considered = cons;
        d.symbols = cplx(prhs[9], &t4);
        d.mod_order = (int32_t)mxGetNumberOfElements(prhs[9]);
        for (d.bits_per_symbol = 0; (1 << d.bits_per_symbol) < d.mod_order; ++d.bits_per_symbol) {}
        d.kappa = mxGetScalar(prhs[10]);
        d.data_div = mxGetScalar(prhs[11]);
        d.despread = (int32_t)mxGetScalar(prhs[12]);
        d.real_detect = (int32_t)mxGetScalar(prhs[13]);
        d.bits_slot = (int32_t)mxGetScalar(prhs[14]);
        d.pilot_slot = (int32_t)mxGetScalar(prhs[15]);
        check(dsce_add_scheme(g_ctx, &d, &id), "dsce_add_scheme");
        plhs[0] = mxCreateDoubleScalar(id + 1);
        mxFree(pil); mxFree(dat); mxFree(cons);
        if (t1) mxDestroyArray(t1);
        if (t2) mxDestroyArray(t2);
        if (t3) mxDestroyArray(t3);
        if (t4) mxDestroyArray(t4);
    } else if (!strcmp(cmd, "build_mmse")) {
        check(dsce_build_mmse(g_ctx, mxGetScalar(prhs[1])), "dsce_build_mmse");
    } else if (!strcmp(cmd, "run")) {
        /* counts are C-ordered [scheme][csi][edge][snr][stage]: reversed dims in MATLAB */
        mwSize dims[5];
        int32_t nsch = (int32_t)mxGetScalar(prhs[4]), nsnr = (int32_t)mxGetScalar(prhs[5]),
                nst = (int32_t)mxGetScalar(prhs[6]);
        dims[0] = nst; dims[1] = nsnr; dims[2] = 2; dims[3] = 2; dims[4] = nsch;
        plhs[0] = mxCreateNumericArray(5, dims, mxINT64_CLASS, mxREAL);
        check(dsce_run(g_ctx, (uint64_t)mxGetScalar(prhs[1]), (uint64_t)mxGetScalar(prhs[2]),
                       (uint64_t)mxGetScalar(prhs[3]), (int64_t*)mxGetInt64s(plhs[0])), "dsce_run");
    } else if (!strcmp(cmd, "channel_realise")) {
        plhs[0] = mxCreateDoubleMatrix((mwSize)mxGetScalar(prhs[3]), (mwSize)mxGetScalar(prhs[4]), mxCOMPLEX);
        check(dsce_channel_realise(g_ctx, (uint64_t)mxGetScalar(prhs[1]), (uint64_t)mxGetScalar(prhs[2]),
                                   (double*)mxGetComplexDoubles(plhs[0])), "dsce_channel_realise");
    } else if (!strcmp(cmd, "get_W")) {
        plhs[0] = mxCreateDoubleMatrix((mwSize)mxGetScalar(prhs[4]), 1, mxCOMPLEX);
        check(dsce_get_W(g_ctx, (int32_t)mxGetScalar(prhs[1]) - 1, (int32_t)mxGetScalar(prhs[2]) - 1,
                         (int32_t)mxGetScalar(prhs[3]), (double*)mxGetComplexDoubles(plhs[0])), "dsce_get_W");
    } else if (!strcmp(cmd, "mmse_onetap")) {
        /* h = dsce_mex('mmse_onetap', id, snrIndex, variant, hP_LS [, LK]) */
        mxArray* t = NULL;
        const int32_t n = 1;
        const mwSize lk = nrhs > 5 ? (mwSize)mxGetScalar(prhs[5]) : 0;
        plhs[0] = mxCreateDoubleMatrix(lk, 1, mxCOMPLEX);
        check(dsce_mmse_onetap(g_ctx, (int32_t)mxGetScalar(prhs[1]) - 1, (int32_t)mxGetScalar(prhs[2]) - 1,
                               (int32_t)mxGetScalar(prhs[3]), cplx(prhs[4], &t), n,
                               (double*)mxGetComplexDoubles(plhs[0])), "dsce_mmse_onetap");
        if (t) mxDestroyArray(t);
    } else if (!strcmp(cmd, "set_noise_slot")) {
        /* dsce_mex('set_noise_slot', id, slot)  (SimpleVersion_DoublyFlat.m:125-126) */
        check(dsce_set_noise_slot(g_ctx, (int32_t)mxGetScalar(prhs[1]) - 1, (int32_t)mxGetScalar(prhs[2])),
              "dsce_set_noise_slot");
    } else if (!strcmp(cmd, "set_interpolation")) {
        /* dsce_mex('set_interpolation', id, I): I = LK x NP weights of a
           PilotSymbolAidedChannelEstimation ('linear', 'MovingBlockAverage', ...),
           e.g. obtained by applying ChannelInterpolation to the NP unit vectors */
        mxArray* t = NULL;
        check(dsce_set_interpolation(g_ctx, (int32_t)mxGetScalar(prhs[1]) - 1, cplx(prhs[2], &t)),
              "dsce_set_interpolation");
        if (t) mxDestroyArray(t);
    } else {
        mexErrMsgIdAndTxt("dsce:usage", "unknown command '%s'", cmd);
    }
}
#endif /* MATLAB_MEX_FILE */
