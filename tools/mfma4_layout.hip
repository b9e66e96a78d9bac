// Layout probe for v_mfma_f64_4x4x4_4b_f64 on gfx950: with A one-hot at lane j and
// B[l] = 1000 + l, D[l] = B[lane_b] for every output lane l that A lane j feeds,
// which reveals the operand / output lane maps.  Prints, per A lane j, the
// (output lane, B lane) pairs.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    D[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[l], B[l], 0.0, 0, 0, 0);
}
int main() {
    double A[64], B[64], D[64];
    double *dA, *dB, *dD;
    (void)hipMalloc(&dA, sizeof A); (void)hipMalloc(&dB, sizeof B); (void)hipMalloc(&dD, sizeof D);
    for (int l = 0; l < 64; ++l) B[l] = 1000 + l;
    (void)hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    for (int j = 0; j < 64; ++j) {
        for (int l = 0; l < 64; ++l) A[l] = l == j ? 1.0 : 0.0;
        (void)hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
        (void)hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
        printf("A%02d:", j);
        for (int l = 0; l < 64; ++l)
            if (D[l] != 0) printf(" D%02d<-B%02d", l, (int)(D[l] - 1000));
        printf("\n");
    }
    return 0;
}
