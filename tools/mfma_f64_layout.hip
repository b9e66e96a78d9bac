// Layout probe for v_mfma_f64_16x16x4_f64 on gfx950 (A = 16x4, B = 4x16, D = 16x16).
// Asymmetric integer data; compares against a host GEMM.  Prints PASS/FAIL.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* D) {
    int l = threadIdx.x;
    double a = A[(l & 15) * 4 + (l >> 4)];      // A[i=l&15][k=l>>4]
    double b = B[(l >> 4) * 16 + (l & 15)];     // B[k=l>>4][j=l&15]
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = c[r];   // D[i][j]
}
int main() {
    double A[64], B[64], D[256], R[256];
    for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = i * 7 + k * 3 + 1;
    for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (k + 1) * (j * j + 2) - 5 * k;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { double s = 0; for (int k = 0; k < 4; ++k) s += A[i*4+k]*B[k*16+j]; R[i*16+j] = s; }
    double *dA, *dB, *dD;
    hipMalloc(&dA, sizeof A); hipMalloc(&dB, sizeof B); hipMalloc(&dD, sizeof D);
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 256; ++i) bad += D[i] != R[i];
    printf("%s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
    return bad != 0;
}
