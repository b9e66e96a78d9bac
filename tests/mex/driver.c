/* TEST-ONLY driver: calls the gateway's mexFunction like MATLAB would and
 * prints, per case, OK + output sizes or the error identifier. */
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
static mxArray* M(size_t m, size_t n, int cplx) {
    mxArray* a = mxCreateDoubleMatrix(m, n, cplx ? mxCOMPLEX : mxREAL);
    double* p = a->data;
    for (size_t i = 0; i < m * n * (cplx ? 2 : 1); ++i) p[i] = 1.0 + (double)(i % 7);
    return a;
}
static mxArray* Lg(size_t n) {
    mxArray* a = mxCreateDoubleMatrix(n, 1, mxREAL);
    free(a->data);
    a->cls = mxLOGICAL_CLASS;
    a->data = calloc(n, 1);
    return a;
}

static void call(const char* tag, int nlhs, int nrhs, mxArray** in) {
    mxArray* out[2] = {NULL, NULL};
    printf("%s:\n", tag);
    if (setjmp(g_err_jmp)) {
        printf("%s -> ERR %s\n", tag, g_err_id);
        return;
    }
    mexFunction(nlhs, out, nrhs, (const mxArray**)in);
    if (out[0])
        printf("%s -> OK %zux%zu\n", tag, mxGetM(out[0]), mxGetN(out[0]));
    else
        printf("%s -> OK\n", tag);
}

int main(void) {
    mxArray* a[20];
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
    a[0] = S("no_such_command");
    call("unknown", 0, 1, a);
    a[0] = S("destroy");
    call("destroy", 0, 1, a);
    a[0] = S("build_mmse");
    call("after_destroy", 0, 1, a);
    return 0;
}
