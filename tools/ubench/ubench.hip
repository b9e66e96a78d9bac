// Issue-cost microbenchmark of the instruction classes in the OFDM chain kernels
// (gfx950): cycles per wave-instruction per SIMD at 1 / 2 / 3 / 4 waves per SIMD,
// 8 independent dependency chains per wave.  tools/ubench/run.sh builds and runs it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void __launch_bounds__(256) k_op(double* out, int n) {
    double a0 = threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    const double b = 1.0000001, c = 1e-9;
    double x0 = a0 * 2, x1 = a1 * 2, x2 = a2 * 2, x3 = a3 * 2, x4 = a4 * 2, x5 = a5 * 2, x6 = a6 * 2, x7 = a7 * 2;
    int i0 = threadIdx.x, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3, i4 = i0 + 4, i5 = i0 + 5, i6 = i0 + 6, i7 = i0 + 7;
    const unsigned long long m = (blockIdx.x & 1) ? 0x5555555555555555ull : 0xaaaaaaaaaaaaaaaaull;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (OP == 0) {
#define F(k) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a##k) : "v"(b), "v"(c));
                REP8(F)
#undef F
            } else if constexpr (OP == 1) {
#define F(k) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a##k) : "v"(c));
                REP8(F)
#undef F
            } else if constexpr (OP == 2) {
#define F(k) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a##k) : "v"(b));
                REP8(F)
#undef F
            } else if constexpr (OP == 3) {
#define F(k) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(i##k));
                REP8(F)
#undef F
            } else if constexpr (OP == 4) {
#define F(k) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(i##k) : "v"(i0), "s"(m));
                REP8(F)
#undef F
            } else if constexpr (OP == 5) {
#define F(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(i##k) : "v"(i0));
                REP8(F)
#undef F
            } else if constexpr (OP == 6) {
#define F(k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(i##k) : "v"(1.0f), "v"(1e-9f));
                REP8(F)
#undef F
            } else if constexpr (OP == 8) {
                // ds_swizzle quad-perm [1,0,3,2], 8 in flight, then wait
#define F(k) asm volatile("ds_swizzle_b32 %0, %0 offset:0x80b1" : "+v"(i##k));
                REP8(F)
#undef F
                asm volatile("s_waitcnt lgkmcnt(0)");
            } else if constexpr (OP == 9) {
                // 8 f64 FMAs beside 8 swizzles (per pair)
#define F(k) asm volatile("v_fma_f64 %0, %0, %2, %3\n ds_swizzle_b32 %1, %1 offset:0x80b1" : "+v"(a##k), "+v"(i##k) : "v"(b), "v"(c));
                REP8(F)
#undef F
                asm volatile("s_waitcnt lgkmcnt(0)");
            } else if constexpr (OP == 10) {
                // v_mfma_f64_4x4x4f64, 8 independent accumulators
#define F(k) a##k = __builtin_amdgcn_mfma_f64_4x4x4f64(b, c, a##k, 0, 0, 0);
                REP8(F)
#undef F
            } else if constexpr (OP == 11) {
                // v_mfma_f64_16x16x4f64 (4 accumulator registers each; 8 chains)
                typedef double d4v __attribute__((ext_vector_type(4)));
                d4v q0 = {a0, a1, a2, a3}, q1 = {a4, a5, a6, a7};
#define F(k) q##k = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, q##k, 0, 0, 0);
                F(0) F(1) F(0) F(1) F(0) F(1) F(0) F(1)
#undef F
                a0 = q0[0]; a1 = q0[1]; a2 = q0[2]; a3 = q0[3]; a4 = q1[0]; a5 = q1[1]; a6 = q1[2]; a7 = q1[3];
            } else if constexpr (OP == 12) {
                // a 4x4x4 MFMA beside 4 independent f64 FMAs
#define F(k) a##k = __builtin_amdgcn_mfma_f64_4x4x4f64(b, c, a##k, 0, 0, 0); \
             asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x##k) : "v"(b), "v"(c));
                REP8(F)
#undef F
            } else if constexpr (OP == 7) {
                // f64 FMA and DPP alternating (the chain network's mix)
#define F(k) asm volatile("v_fma_f64 %0, %0, %2, %3\n v_mov_b32_dpp %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a##k), "+v"(i##k) : "v"(b), "v"(c));
                REP8(F)
#undef F
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + i0 + i1 + i2 + i3 + i4 + i5 + i6 + i7;
}

template <int OP>
static float run(double* d, int blocks, int n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, n);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double ghz = p.clockRate / 1e6;
    double* d;
    hipMalloc(&d, (size_t)cus * 8 * 256 * sizeof(double));
    const char* names[] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_mov_b32_dpp", "v_cndmask_b32", "v_add_u32",
                           "v_fma_f32", "fma_f64+dpp (per pair)", "ds_swizzle_b32 (8, wait)",
                           "fma_f64+swizzle (per pair)", "mfma_f64_4x4x4", "mfma_f64_16x16x4 (2 chains)",
                           "mfma4x4x4+fma_f64 (per pair)"};
    const int n = 2000;
    printf("CUs %d clock %.2f GHz; cycles per wave-instruction per SIMD (8 chains per wave)\n", cus, ghz);
    printf("%-24s %8s %8s %8s %8s\n", "op", "1 w/SIMD", "2", "3", "4");
    for (int op = 0; op < 13; ++op) {
        printf("%-24s", names[op]);
        for (int w = 1; w <= 4; ++w) {
            const int blocks = cus * w;          // 256 threads = one wave per SIMD per block
            float ms = 0;
            switch (op) {
                case 0: ms = run<0>(d, blocks, n); break;
                case 1: ms = run<1>(d, blocks, n); break;
                case 2: ms = run<2>(d, blocks, n); break;
                case 3: ms = run<3>(d, blocks, n); break;
                case 4: ms = run<4>(d, blocks, n); break;
                case 5: ms = run<5>(d, blocks, n); break;
                case 6: ms = run<6>(d, blocks, n); break;
                case 7: ms = run<7>(d, blocks, n); break;
                case 8: ms = run<8>(d, blocks, n); break;
                case 9: ms = run<9>(d, blocks, n); break;
                case 10: ms = run<10>(d, blocks, n); break;
                case 11: ms = run<11>(d, blocks, n); break;
                case 12: ms = run<12>(d, blocks, n); break;
            }
            const double instr_per_simd = (double)w * n * 32;      // per wave: n x 4 x 8
            printf(" %8.2f", ms * 1e-3 * ghz * 1e9 / instr_per_simd);
        }
        printf("\n");
    }
    hipFree(d);
    return 0;
}
