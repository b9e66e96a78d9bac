// Layout probe: per-unit vectors [row][U] (unit fastest, row stride U*16 B) vs
// blocked [unit/64][row][64]; read-modify-write of LK rows per unit, RB rows per
// wave, with the stage kernel's launch shape.  Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct c2 { double x, y; };

template <int RB, bool BLOCKED>
__global__ void __launch_bounds__(256) k_rmw(const double2* __restrict__ in, double2* __restrict__ out, int U, int LK, int nrb) {
    const int rbk = blockIdx.x % nrb, ug = blockIdx.x / nrb;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ub = ug * 4 + wv;                       // 64-unit group
    double2 v[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int row = rbk * RB + r;
        const size_t i = BLOCKED ? ((size_t)ub * LK + row) * 64 + lane : (size_t)row * U + ub * 64 + lane;
        v[r] = in[i];
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int row = rbk * RB + r;
        const size_t i = BLOCKED ? ((size_t)ub * LK + row) * 64 + lane : (size_t)row * U + ub * 64 + lane;
        out[i] = make_double2(v[r].x * 2.0, v[r].y + 1.0);
    }
}

template <int RB, bool BLOCKED>
float run(const double2* in, double2* out, int U, int LK) {
    const int nrb = LK / RB;
    dim3 grid((U / 256) * nrb);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_rmw<RB, BLOCKED><<<grid, 256>>>(in, out, U, LK, nrb);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) k_rmw<RB, BLOCKED><<<grid, 256>>>(in, out, U, LK, nrb);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main() {
    const int U = 114688, LK = 336;
    const size_t n = (size_t)U * LK;
    double2 *in, *out;
    hipMalloc(&in, n * sizeof(double2));
    hipMalloc(&out, n * sizeof(double2));
    hipMemset(in, 0, n * sizeof(double2));
    const double gb = 2.0 * n * sizeof(double2) / 1e9;
    float t;
    t = run<8, false>(in, out, U, LK); printf("strided RB=8   %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    t = run<8, true>(in, out, U, LK);  printf("blocked RB=8   %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    t = run<16, false>(in, out, U, LK); printf("strided RB=16  %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    t = run<16, true>(in, out, U, LK);  printf("blocked RB=16  %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    t = run<48, false>(in, out, U, LK); printf("strided RB=48  %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    t = run<48, true>(in, out, U, LK);  printf("blocked RB=48  %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    return 0;
}
