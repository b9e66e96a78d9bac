// Cost of one sample (m) of the DFT-24 chain's 4-point network across the four
// time quarters of a unit, per wave, two ways (gfx950):
//   dpp : k_pic_fft's network (lane twiddle c_mulf, DPP xor2, FMAs, +-i lane
//         select, DPP xor1, FMAs) with a unit on a lane quad
//   mfma: the quarters on the four 16-lane rows, DFT-4 (twiddle folded into the
//         per-sample A operand) as four v_mfma_f64_4x4x4f64 (re/im x two K halves)
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/ubench/net.hip -o tools/ubench/net
// (on the box: tools/ubench/net > gpurun_out/net.txt; result in profiles/r03k_ubench_network.txt)
// 8 independent chains per wave, cycles per chain-step per SIMD at 1..4 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int hi = __double2hiint(v), lo = __double2loint(v);
    return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, CTRL, 0xf, 0xf, false),
                            __builtin_amdgcn_mov_dpp(lo, CTRL, 0xf, 0xf, false));
}

template <int MODE>
__global__ void __launch_bounds__(256) k_net(double* out, int n, double2 tw, double2 aa) {
    const int l = threadIdx.x & 63, r = l & 3;
    const double sg1 = (r >> 1) ? -1.0 : 1.0, sg2 = (r & 1) ? -1.0 : 1.0;
    double xr[8], xi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        xr[k] = 1e-3 * threadIdx.x + k;
        xi[k] = 2e-3 * threadIdx.x - k;
    }
    const double ar = aa.x, ai = aa.y, nai = -aa.y;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (MODE == 0) {
                // p = x * tw, e = sg1 p + xor2(p), e *= (r == 3 ? i : 1), t = sg2 e + xor1(e)
                const double px = fma(xr[k], tw.x, -(xi[k] * tw.y)), py = fma(xr[k], tw.y, xi[k] * tw.x);
                const double vx = dpp_d<0x4e>(px), vy = dpp_d<0x4e>(py);
                double ex = fma(sg1, px, vx), ey = fma(sg1, py, vy);
                const double nx = -ey, ny = ex;
                ex = r == 3 ? nx : ex;
                ey = r == 3 ? ny : ey;
                const double qx = dpp_d<0xb1>(ex), qy = dpp_d<0xb1>(ey);
                xr[k] = fma(sg2, ex, qx);
                xi[k] = fma(sg2, ey, qy);
            } else {
                double dr = __builtin_amdgcn_mfma_f64_4x4x4f64(ar, xr[k], 0.0, 0, 0, 0);
                dr = __builtin_amdgcn_mfma_f64_4x4x4f64(nai, xi[k], dr, 0, 0, 0);
                double di = __builtin_amdgcn_mfma_f64_4x4x4f64(ar, xi[k], 0.0, 0, 0, 0);
                di = __builtin_amdgcn_mfma_f64_4x4x4f64(ai, xr[k], di, 0, 0, 0);
                xr[k] = dr;
                xi[k] = di;
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += xr[k] + xi[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
static float run(double* d, int blocks, int n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double2 tw = make_double2(0.96592582628906829, 0.25881904510252076), aa = make_double2(0.5, 0.25);
    hipLaunchKernelGGL(k_net<MODE>, dim3(blocks), dim3(256), 0, 0, d, n, tw, aa);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_net<MODE>, dim3(blocks), dim3(256), 0, 0, d, n, tw, aa);
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
    const int n = 2000;
    printf("CUs %d clock %.2f GHz; cycles per network sample (m) per wave per SIMD\n", cus, ghz);
    printf("%-28s %8s %8s %8s %8s\n", "variant", "1 w/SIMD", "2", "3", "4");
    const char* names[] = {"dpp network (k_pic_fft)", "4 x mfma_f64_4x4x4"};
    for (int mode = 0; mode < 2; ++mode) {
        printf("%-28s", names[mode]);
        for (int w = 1; w <= 4; ++w) {
            const int blocks = cus * w;
            const float ms = mode ? run<1>(d, blocks, n) : run<0>(d, blocks, n);
            printf(" %8.2f", ms * 1e-3 * ghz * 1e9 / ((double)w * n * 8));
        }
        printf("\n");
    }
    hipFree(d);
    return 0;
}
