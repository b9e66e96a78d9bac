/* TEST-ONLY driver: calls the gateway's mexFunction like MATLAB would and
 * prints, per case, OK + output sizes or the error identifier.
 *   drv                       the fixed case list below
 *   drv replay cmd:nrhs:nlhs ...
 *                             one call per triple, with default arguments of the
 *                             right class and size for each argument position
 *                             (tests/test_mex_gateway.py replays every
 *                             dsce_mex(...) call of INTEGRATION.md this way) */
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

extern jmp_buf g_err_jmp;
extern char g_err_id[64];
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

static mxArray* S(const char* s) {
    mxArray* a = mxCreateDoubleMatrix(1, strlen(s), mxREAL);
    free(a->data);
    a->data = calloc(1, 1);
    a->cls = mxCHAR_CLASS;
    a->str = strdup(s);
    return a;
}
static mxArray* D(double v) { return mxCreateDoubleScalar(v); }
/* element i = (1 + i % 7) - (1 + i % 5) j, or 1 + i % 7 when real (mex_stub.c checks
 * that the ABI receives exactly these values, interleaved) */
static mxArray* M(size_t m, size_t n, int cplx) {
    mxArray* a = mxCreateDoubleMatrix(m, n, cplx ? mxCOMPLEX : mxREAL);
    for (size_t i = 0; i < m * n; ++i) tst_set_c(a, i, 1.0 + (double)(i % 7), cplx ? -(1.0 + (double)(i % 5)) : 0.0);
    return a;
}
static mxArray* Lg(size_t n) {
    mxArray* a = mxCreateDoubleMatrix(n, 1, mxREAL);
    free(a->data);
    a->cls = mxLOGICAL_CLASS;
    a->data = calloc(n, 1);
    return a;
}

/* Modulation.OFDM / Modulation.FBMC objects with the properties dsce_mex's
 * tx_matrices reads (OFDM.m:53-88, FBMC.m:61-160 field names; C2 / C3 values) */
static mxArray* St(int n, const char* const* nm, mxArray** v) { return tst_struct(n, nm, v); }
static mxArray* ofdm_object(int real_signal) {
    const char* nn[] = {"Subcarriers", "MCSymbols", "SamplesTotal"};
    mxArray* nv[] = {D(24), D(14), D(540)};
    const char* pn[] = {"TransmitRealSignal", "SubcarrierSpacing", "SamplingRate"};
    mxArray* pv[] = {D(real_signal), D(15e3), D(360e3)};
    const char* in[] = {"FFTSize", "IntermediateFrequency", "TimeSpacing", "NormalizationFactor", "CyclicPrefix",
                        "ZeroGuardSamples"};
    mxArray* iv[] = {D(24), D(0), D(26), D(1.0), D(2), D(88)};
    const char* on[] = {"Nr", "PHY", "Implementation"};
    mxArray* ov[] = {St(3, nn, nv), St(3, pn, pv), St(6, in, iv)};
    return tst_object("Modulation.OFDM", 3, on, ov);
}
static mxArray* fbmc_object(const char* method) {
    const char* nn[] = {"Subcarriers", "MCSymbols", "SamplesTotal"};
    mxArray* nv[] = {D(24), D(30), D(540)};
    const char* pn[] = {"TransmitRealSignal", "SubcarrierSpacing", "SamplingRate", "TimeSpacing"};
    mxArray* pv[] = {D(0), D(15e3), D(360e3), D(12.0 / 360e3)};
    const char* in[] = {"FFTSize", "IntermediateFrequency", "TimeSpacing", "NormalizationFactor", "InitialPhaseShift"};
    mxArray* iv[] = {D(24), D(0), D(12), D(1.0), D(0)};
    const char* fn[] = {"TimeDomain"};
    mxArray* fv[] = {M(192, 1, 0)};
    const char* on[] = {"Nr", "PHY", "Implementation", "PrototypeFilter", "Method"};
    mxArray* ov[] = {St(3, nn, nv), St(4, pn, pv), St(5, in, iv), St(1, fn, fv), S(method)};
    return tst_object("Modulation.FBMC", 5, on, ov);
}

static mxArray* g_last_out;

static void call(const char* tag, int nlhs, int nrhs, mxArray** in) {
    mxArray* out[2] = {NULL, NULL};
    printf("%s:\n", tag);
    g_last_out = NULL;
    if (setjmp(g_err_jmp)) {
        printf("%s -> ERR %s\n", tag, g_err_id);
        return;
    }
    mexFunction(nlhs, out, nrhs, (const mxArray**)in);
    g_last_out = out[0];
    if (out[0])
        printf("%s -> OK %zux%zu\n", tag, mxGetM(out[0]), mxGetN(out[0]));
    else
        printf("%s -> OK\n", tag);
}

/* the complex outputs the stub writes: channel_realise element k = 2k + (2k+1) j;
 * mmse_onetap element k = (a + 2k) - (k + 0.25) j with a = the input sum */
static void check_out(const char* tag, int which) {
    int ok = g_last_out != NULL && mxIsComplex(g_last_out);
    double a0 = 0.0;
    for (size_t k = 0; ok && k < mxGetNumberOfElements(g_last_out); ++k) {
        double re, im;
        tst_get_c(g_last_out, k, &re, &im);
        if (k == 0) a0 = re;
        if (which == 0) ok = re == 2.0 * k && im == 2.0 * k + 1;
        else ok = im == -0.5 * (2.0 * k + 1) && re - 2.0 * k == a0;
    }
    printf("check %s output %s\n", tag, ok ? "OK" : "BAD");
}

/* default argument `pos` of command `cmd` (replay mode): the class and size the
 * gateway expects, for the stub engine's dimensions (mex_stub.c) */
static mxArray* S(const char* s);
static mxArray* Lg(size_t n);
static mxArray* default_arg(const char* cmd, int pos) {
    if (pos == 0) return S(cmd);
    if (!strcmp(cmd, "create")) {
        /* a device vector [0 1 ... 7] (dsce_create_multi) */
        mxArray* v = mxCreateDoubleMatrix(1, 8, mxREAL);
        for (size_t i = 0; i < 8; ++i) tst_set_c(v, i, (double)i, 0.0);
        return v;
    }
    if (!strcmp(cmd, "set_channel")) {
        const double v[7] = {0, 360e3, 0, 540, 1158.2, 200, 0};
        return pos == 2 ? M(2, 1, 0) : D(v[pos < 7 ? pos : 0]);
    }
    if (!strcmp(cmd, "set_snr")) return pos == 1 ? M(7, 1, 0) : D(4);
    if (!strcmp(cmd, "add_scheme")) {
        switch (pos) {
            case 1: return D(24);
            case 2: return D(14);
            case 3: case 4: return M(540, 336, 1);
            case 5: return M(336, 336, 0);
            case 6: return M(16, 1, 0);
            case 7: return M(320, 1, 0);
            case 8: return Lg(320);
            case 9: return M(256, 1, 1);
            case 10: return D(2.1);
            case 11: return D(1.02);
            case 14: return D(2);
            case 15: return D(1);
            default: return D(0);
        }
    }
    if (!strcmp(cmd, "build_mmse")) return D(1e-8);
    if (!strcmp(cmd, "set_batch")) return D(8192);
    if (!strcmp(cmd, "run")) return D(pos == 3 ? 25 : pos == 1 ? 1 : 0);
    if (!strcmp(cmd, "channel_realise")) return D(pos == 1 ? 1 : 3);
    if (!strcmp(cmd, "get_W")) return D(pos == 3 ? 0 : 1);
    if (!strcmp(cmd, "mmse_onetap")) return pos == 4 ? M(16, 1, 1) : D(pos == 2 ? 4 : pos == 3 ? 0 : 1);
    if (!strcmp(cmd, "set_noise_slot")) return D(pos == 1 ? 1 : 0);
    if (!strcmp(cmd, "set_interpolation")) return pos == 2 ? M(336, 16, 0) : D(1);
    if (!strcmp(cmd, "set_option")) return pos == 1 ? S("xcd") : D(1);
    if (!strcmp(cmd, "tx_matrices")) return ofdm_object(0);
    if (!strcmp(cmd, "enable_mse")) return D(1);
    return D(1);   /* bits_per_rep, scheme_dims, path_info: scheme id 1 */
}

static int replay(int argc, char** argv) {
    for (int i = 2; i < argc; ++i) {
        char cmd[64];
        int nrhs = 0, nlhs = 0;
        mxArray* a[24];
        if (sscanf(argv[i], "%63[^:]:%d:%d", cmd, &nrhs, &nlhs) != 3 || nrhs < 1 || nrhs > 24) {
            printf("replay %s -> ERR parse\n", argv[i]);
            continue;
        }
        for (int k = 0; k < nrhs; ++k) a[k] = default_arg(cmd, k);
        call(argv[i], nlhs, nrhs, a);
    }
    return 0;
}

int main(int argc, char** argv) {
    mxArray* a[20];
    if (argc > 1 && !strcmp(argv[1], "replay")) return replay(argc, argv);
    a[0] = S("run"); a[1] = D(1); a[2] = D(0); a[3] = D(64);
    call("run_before_create", 1, 4, a);
    a[0] = S("create");
    call("create", 0, 1, a);
    a[0] = S("run");
    call("run", 1, 4, a);
    a[4] = D(1); a[5] = D(7); a[6] = D(5);
    call("run_old_7_args", 1, 7, a);
    a[0] = S("mmse_onetap"); a[1] = D(1); a[2] = D(4); a[3] = D(0); a[4] = M(16, 1, 1);
    call("mmse_onetap_documented_5_args", 1, 5, a);
    check_out("mmse_onetap", 1);
    a[4] = M(16, 3, 0);
    call("mmse_onetap_3_vectors_real", 1, 5, a);
    a[4] = M(15, 1, 1);
    call("mmse_onetap_wrong_np", 1, 5, a);
    call("mmse_onetap_4_args", 1, 4, a);
    a[4] = M(16, 1, 1); a[5] = D(336);
    call("mmse_onetap_old_6_args", 1, 6, a);
    a[0] = S("get_W"); a[1] = D(1); a[2] = D(1); a[3] = D(0);
    call("get_W", 1, 4, a);
    a[4] = D(100);
    call("get_W_old_5_args", 1, 5, a);
    a[1] = D(0);
    call("get_W_scheme_0", 1, 4, a);
    a[0] = S("channel_realise"); a[1] = D(1); a[2] = D(3);
    call("channel_realise", 1, 3, a);
    check_out("channel_realise", 0);
    a[3] = D(540); a[4] = D(2);
    call("channel_realise_old_5_args", 1, 5, a);
    a[0] = S("add_scheme"); a[1] = D(24); a[2] = D(14); a[3] = M(540, 336, 1); a[4] = M(540, 336, 1);
    a[5] = M(336, 336, 0); a[6] = M(16, 1, 0); a[7] = M(320, 1, 0); a[8] = Lg(320); a[9] = M(256, 1, 1);
    a[10] = D(2.1); a[11] = D(1.02); a[12] = D(0); a[13] = D(0); a[14] = D(2); a[15] = D(1);
    call("add_scheme", 1, 16, a);
    a[4] = M(540, 335, 1);
    call("add_scheme_bad_Q", 1, 16, a);
    a[4] = M(540, 336, 1); a[7] = M(319, 1, 0);
    call("add_scheme_bad_dataIdx", 1, 16, a);
    call("add_scheme_15_args", 1, 15, a);
    a[0] = S("set_interpolation"); a[1] = D(1); a[2] = M(336, 16, 0);
    call("set_interpolation", 0, 3, a);
    a[2] = M(336, 15, 0);
    call("set_interpolation_bad", 0, 3, a);
    a[0] = S("set_option"); a[1] = S("xcd"); a[2] = D(0);
    call("set_option", 0, 3, a);
    a[1] = D(3);
    call("set_option_bad_name", 0, 3, a);
    a[0] = S("scheme_dims"); a[1] = D(1);
    call("scheme_dims", 1, 2, a);
    call("scheme_dims_2_outputs", 2, 2, a);
    a[0] = S("set_channel"); a[1] = D(360e3); a[2] = M(2, 1, 0); a[3] = D(540); a[4] = D(1158.2); a[5] = D(200);
    a[6] = D(0);
    call("set_channel", 0, 7, a);
    a[3] = D(540.5);
    call("set_channel_fractional_N", 0, 7, a);
    a[0] = S("tx_matrices"); a[1] = ofdm_object(0);
    call("tx_matrices_ofdm", 2, 2, a);
    check_out("tx_matrices", 0);
    a[1] = fbmc_object("Hermite-OQAM");
    call("tx_matrices_fbmc", 1, 2, a);
    check_out("tx_matrices_fbmc", 0);
    a[1] = D(1);
    call("tx_matrices_not_object", 1, 2, a);
    a[1] = ofdm_object(1);
    call("tx_matrices_real_signal", 2, 2, a);
    a[1] = fbmc_object("PHYDYAS-OQAM");
    call("tx_matrices_phydyas", 1, 2, a);
    a[1] = ofdm_object(0);
    call("tx_matrices_3_outputs", 3, 2, a);
    a[0] = S("enable_mse"); a[1] = D(1);
    call("enable_mse", 0, 2, a);
    a[0] = S("get_mse");
    call("get_mse", 2, 1, a);
    call("get_mse_extra_arg", 2, 2, a);
    a[0] = S("structured_check"); a[1] = D(1);
    call("structured_check", 1, 2, a);
    a[0] = S("group_info");
    call("group_info_single", 2, 1, a);
    a[0] = S("create"); a[1] = M(1, 8, 0);
    call("create_multi_8", 0, 2, a);        /* devices 1 + i % 7: device 1 repeats -> host sum */
    a[0] = S("group_info");
    call("group_info_multi", 2, 1, a);
    a[0] = S("run"); a[1] = D(1); a[2] = D(0); a[3] = D(64);
    call("run_multi", 1, 4, a);
    a[0] = S("create"); a[1] = M(0, 0, 0);
    call("create_empty_devices", 0, 2, a);
    a[0] = S("create"); a[1] = D(0);
    call("create_again", 0, 2, a);
    a[0] = S("no_such_command");
    call("unknown", 0, 1, a);
    a[0] = S("destroy");
    call("destroy", 0, 1, a);
    a[0] = S("build_mmse");
    call("after_destroy", 0, 1, a);
    return 0;
}
