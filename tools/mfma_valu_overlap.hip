// Does an f64 MFMA overlap with f64 / int VALU work on the same SIMD (gfx950)?
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_valu_overlap.hip -o tools/mfma_valu_overlap
// Kernels (1024 workgroups x 512 threads = 2 waves per SIMD, ITERS iterations):
//   mfma   every wave: 8 independent v_mfma_f64_16x16x4_f64 per iteration
//   fma    every wave: 32 v_fma_f64 per iteration (8 independent chains)
//   iadd   every wave: 32 v_add_u32 per iteration (8 chains)
//   same_f every wave: the mfma and the fma work of one iteration, interleaved
//   split_f waves 0-3 of a workgroup: mfma work, waves 4-7: fma work (x2, so
//           each SIMD gets the same total as same_f)
//   same_i, split_i    the same with v_add_u32 instead of v_fma_f64
// Prints ms per kernel; if the pipes overlap, same/split ~ max(mfma, valu),
// otherwise ~ sum.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 4096;

template <bool DO_MFMA, bool DO_F, bool DO_I, int SPLIT>
__global__ void __launch_bounds__(512) k(double* out, double seed) {
    const int w = threadIdx.x >> 6;
    bool dm = DO_MFMA, df = DO_F, di = DO_I;
    int rep = 1;
    if (SPLIT) {                         // waves 0-3 matrix, 4-7 vector (twice the vector work)
        const bool vec = __builtin_amdgcn_readfirstlane(w) >= 4;
        dm = DO_MFMA && !vec;
        df = DO_F && vec;
        di = DO_I && vec;
        rep = 2;
    }
    d4 acc[8];
    for (int k = 0; k < 8; ++k) acc[k] = (d4){0, 0, 0, 0};
    double f[8];
    unsigned u[8];
    for (int k = 0; k < 8; ++k) {
        f[k] = seed + threadIdx.x * 1e-3 + k;
        u[k] = threadIdx.x + k;
    }
    const double a = seed + 1e-3 * (threadIdx.x & 63), b = 1.0 - 1e-3 * (threadIdx.x & 7);
    for (int i = 0; i < ITERS; ++i) {
        if (dm) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
        }
        for (int r = 0; r < rep; ++r) {
            if (df) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int k = 0; k < 8; ++k) f[k] = fma(f[k], b, a);
            }
            if (di) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int k = 0; k < 8; ++k) u[k] = u[k] * 3u + (unsigned)i;
            }
        }
    }
    double s = 0.0;
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][3] + f[k] + (double)u[k];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <class K>
float timeit(K kern, double* out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(1024), dim3(512), 0, 0, out, 0.5);
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(1024), dim3(512), 0, 0, out, 0.5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}

int main() {
    double* out;
    CHECK(hipMalloc(&out, 1024 * 512 * sizeof(double)));
    printf("mfma    %.3f ms\n", timeit(k<true, false, false, 0>, out));
    printf("fma     %.3f ms\n", timeit(k<false, true, false, 0>, out));
    printf("iadd    %.3f ms\n", timeit(k<false, false, true, 0>, out));
    printf("same_f  %.3f ms\n", timeit(k<true, true, false, 0>, out));
    printf("split_f %.3f ms\n", timeit(k<true, true, false, 1>, out));
    printf("same_i  %.3f ms\n", timeit(k<true, false, true, 0>, out));
    printf("split_i %.3f ms\n", timeit(k<true, false, true, 1>, out));
    CHECK(hipDeviceSynchronize());
    return 0;
}
