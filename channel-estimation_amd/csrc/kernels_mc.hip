// kernels_mc.hip — per-realisation hot path of DoublySelectiveChannelEstimation.m
// (script:350-564) as CDNA4 HIP kernels.
//
// Mapping: one wavefront = 64 lanes = 64 independent units (realisation, or
// realisation x SNR point).  Operators shared by all units (G, Q, P, W,
// constellation) are addressed with wave-uniform indices, so the compiler
// reads them with scalar loads (s_load / s_buffer_load) and broadcasts them to
// the lanes; per-unit vectors live in HBM as [element][unit] and every access
// is a coalesced 16-byte-per-lane vector load.  Complex arithmetic is fp64
// throughout (the reference is fp64 MATLAB).
//
// Compile with -ffp-contract=off: the RNG transforms and the Jakes phase must
// round exactly like the NumPy oracle; explicit fma() is used where fusion is
// wanted (matvec inner loops).
#include "dsce_kernels.h"
#include "bm_tables.h"

#include <math.h>
#include <algorithm>
#include <stdexcept>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

namespace dsce {

static constexpr double TWO_PI = 6.283185307179586;   // 2*pi rounded (== 2.0*np.pi)
static constexpr int WAVE = 64;

// ---------------------------------------------------------------------------
// wave reductions
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Integer wave sum by DPP (quad perms, half-row / row mirrors, row broadcasts)
// instead of six ds_bpermute round trips; every lane returns the total.
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xb1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4e, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);   // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false);   // row_mirror: every lane holds its row's sum
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 into rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Channel-estimation MSE of one stage (build-defined; the reference computes no
// MSE): sum over units and rows of |h_hat - h|^2 (h = diag(D), the perfect-CSI
// one-tap channel) into err[(scheme * nsnr + snr) * nstage + stage], and of
// |h|^2 into pow[scheme * nsnr + snr] at stage 0.  One fp64 atomic per wave.
// valid = false: the lane's unit is a padding realisation of the batch (its
// rep index >= McBuffers::rvalid) and contributes nothing.
__device__ __forceinline__ void flush_mse(double e, double pw, double* err, double* pow, int scheme, int nsnr, int snr,
                                          int nstage, int stage, bool valid) {
    const double te = wave_sum_d(valid ? e : 0.0), tp = wave_sum_d(valid ? pw : 0.0);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&err[((size_t)scheme * nsnr + snr) * nstage + stage], te);
        if (stage == 0) atomicAdd(&pow[(size_t)scheme * nsnr + snr], tp);
    }
}

// Slicer tables staged in LDS (levels and the level-grid -> symbol map are
// gathered per lane; from global memory these gathers were the stage's latency
// chain).  The cell index comes from a multiply by 1/step: an index off by one
// can only occur when x sits (to rounding) on a level, where both candidate
// pairs resolve to that level; ties (mid-points) keep the first-minimum rule.
struct SlicerLds {
    double lvI[16], lvQ[16];
    int grid[256];
};

__device__ __forceinline__ void slicer_load(SlicerLds& t, const SchemeK& sk, int tid, int nthreads) {
    for (int i = tid; i < sk.nI; i += nthreads) t.lvI[i] = sk.lvI[i];
    for (int i = tid; i < sk.nQ; i += nthreads) t.lvQ[i] = sk.lvQ[i];
    for (int i = tid; i < sk.nI * sk.nQ; i += nthreads) t.grid[i] = sk.grid_sym[i];
}

// Constellation + slicer tables into LDS with every global load issued before
// the first LDS write (one memory round trip, not one per table).  NTH threads.
template <int NTH>
__device__ __forceinline__ void stage_tables(double2* sym, SlicerLds& t, const SchemeK& sk, int tid) {
    constexpr int PER = 256 / NTH;                      // entries of the 256-slot tables per thread
    double2 sv[PER];
    int gv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        // Clamped, unconditional loads, masked afterwards: a guarded load becomes a
        // branch with its own vmcnt(0) wait, and the table loads then serialise.
        const int i = tid + k * NTH;
        const double2 a = sk.symbols[min(i, sk.M - 1)];
        const int g = sk.grid_sym[min(i, sk.nI * sk.nQ - 1)];
        sv[k].x = i < sk.M ? a.x : 0.0;
        sv[k].y = i < sk.M ? a.y : 0.0;
        gv[k] = i < sk.nI * sk.nQ ? g : 0;
    }
    const int lt = min(tid, 15);
    const double lia = sk.lvI[min(lt, sk.nI - 1)];
    const double lqa = sk.lvQ[min(lt, sk.nQ - 1)];
    const double li = tid < sk.nI ? lia : 0.0;
    const double lq = tid < sk.nQ ? lqa : 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        sym[tid + k * NTH] = sv[k];
        t.grid[tid + k * NTH] = gv[k];
    }
    if (tid < 16) {
        t.lvI[tid] = li;
        t.lvQ[tid] = lq;
    }
}

// Branch-free (selects only): with branches each row's slicer became a chain of
// exec-mask blocks, every one ending in its own LDS wait, and the rows of an
// epilogue could not be interleaved.
__device__ __forceinline__ int nearest_level_fast(const double* lv, int n, double x, double istep, int& alt) {
    // n == 1 (the Q axis of a real slicer) folds in: i = i1 = 0, no alternative
    int i = (int)floor((x - lv[0]) * istep);
    i = i < 0 ? 0 : (i > n - 2 ? max(n - 2, 0) : i);
    const int i1 = min(i + 1, n - 1);
    const double d0 = fabs(x - lv[i]), d1 = fabs(x - lv[i1]);
    alt = d1 == d0 && i1 != i ? i1 : -1;
    return d1 < d0 ? i1 : i;
}

// nearest grid point; on a tie the smallest symbol index (MATLAB min's first
// index).  The alternative entries are read unconditionally at clamped indices:
// a missing alternative reads the primary entry again, which leaves the min as is.
__device__ __forceinline__ int slice_fast(const SlicerLds& t, int nI, int nQ, double2 z, double sI, double sQ) {
    int aI, aQ;
    const int iI = nearest_level_fast(t.lvI, nI, z.x, sI, aI);
    const int iQ = nearest_level_fast(t.lvQ, nQ, z.y, sQ, aQ);
    const int jI = aI >= 0 ? aI : iI, jQ = aQ >= 0 ? aQ : iQ;
    const int b0 = t.grid[iI * nQ + iQ], b1 = t.grid[jI * nQ + iQ];
    const int b2 = t.grid[iI * nQ + jQ], b3 = t.grid[jI * nQ + jQ];
    return min(min(b0, b1), min(b2, b3));
}

// 1 / x by v_rcp_f64 and two Newton steps (5 instructions; the IEEE division is
// ~10 with its scale / fixup for denormals and overflow, which these operands —
// |h|^2 of a channel estimate — never reach); error ~1 ulp
__device__ __forceinline__ double recip_fast(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
// a / b with one fast reciprocal
__device__ __forceinline__ double2 c_div_fast(double2 a, double2 b) {
    const double id = recip_fast(b.x * b.x + b.y * b.y);
    return make_double2((a.x * b.x + a.y * b.y) * id, (a.y * b.x - a.x * b.y) * id);
}
// a / b with one division (rounding-level differences to c_div)
__device__ __forceinline__ double2 c_div1(double2 a, double2 b) {
    const double id = 1.0 / (b.x * b.x + b.y * b.y);
    return make_double2((a.x * b.x + a.y * b.y) * id, (a.y * b.x - a.x * b.y) * id);
}

// Error counters of one wave: cnt[csi*2 + edge] summed over the wave and added
// with ONE atomic instruction (lanes 0-3 carry the four totals) instead of four
// single-lane atomics; device-scope atomics are issued per wave-instruction, so
// this is 4x fewer of them.  base = counter index of (scheme, csi 0, edge 0,
// snr, stage); stride_edge = nsnr * nstage; ncsi = 1 skips the perfect-CSI pair.
// valid: as flush_mse.
__device__ __forceinline__ void flush_counts(const int (&cnt)[4], unsigned long long* counters, size_t base,
                                             size_t stride_edge, int ncsi, bool valid) {
    int t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = wave_sum(valid ? cnt[k] : 0);
    const int l = threadIdx.x & 63;
    if (l < 2 * ncsi) {
        const int v = l == 0 ? t[0] : l == 1 ? t[1] : l == 2 ? t[2] : t[3];
        const int csi = l >> 1, edge = l & 1;
        if (v) atomicAdd(&counters[base + (size_t)(csi * 2 + edge) * stride_edge], (unsigned long long)v);
    }
}

// ---------------------------------------------------------------------------
// a2: Jakes / Uniform sum-of-sinusoids impulse response, FastFading.m:222-238.
// IR[n, tap] = sqrt(PDPn) / sqrt(Paths) * sum_p exp(j 2 pi (phi_p + fD_p n dt)).
// Block 256 = 4 waves = 4 realisations of one tap; each wave draws its
// realisation's 2 x Paths random numbers (Philox, THETA/PHI streams) into LDS
// together with the per-path rotation w_p = exp(j 2 pi fD_p dt).  A lane owns
// JCH consecutive samples: one exact sincos per path at the chunk start, then
// the three-term recurrence below (|error| <~ JCH^2 * 1e-16, far inside the
// 1e-12 parity tolerance).  grid (ceil(nchunk/64), R/4, ntap).
// Output IR[tap][n][rep] (only the non-zero-power taps).
// ---------------------------------------------------------------------------
// (cos, sin)(2 pi x) for |x| of a few turns: quarter-turn reduction (exact),
// then Taylor polynomials on |theta| <= pi/4 (truncation < 1e-16); ~25 FP64
// instructions instead of the general-argument library sincos.
__device__ __forceinline__ double2 cis_turns(double x) {
    const double k = rint(4.0 * x);
    const double r = fma(-0.25, k, x);                      // exact: |r| <= 1/8
    const double t = TWO_PI * r, t2 = t * t;
    double sp = 1.0 / 1307674368000.0;                      // 1/15!
    sp = fma(sp, -t2, 1.0 / 6227020800.0);
    sp = fma(sp, -t2, 1.0 / 39916800.0);
    sp = fma(sp, -t2, 1.0 / 362880.0);
    sp = fma(sp, -t2, 1.0 / 5040.0);
    sp = fma(sp, -t2, 1.0 / 120.0);
    sp = fma(sp, -t2, 1.0 / 6.0);
    const double sn = fma(-t * t2, sp, t);
    double cp = 1.0 / 20922789888000.0;                     // 1/16!
    cp = fma(cp, -t2, 1.0 / 87178291200.0);
    cp = fma(cp, -t2, 1.0 / 479001600.0);
    cp = fma(cp, -t2, 1.0 / 3628800.0);
    cp = fma(cp, -t2, 1.0 / 40320.0);
    cp = fma(cp, -t2, 1.0 / 720.0);
    cp = fma(cp, -t2, 1.0 / 24.0);
    cp = fma(cp, -t2, 0.5);
    const double cs = fma(-t2, cp, 1.0);
    // quadrant q: (c, s) = (cs, sn), (-sn, cs), (-cs, -sn), (sn, -cs) -- selects, no branches
    const int q = ((int)k) & 3;
    const double a = (q & 1) ? sn : cs, b = (q & 1) ? cs : sn;
    return make_double2(((q + 1) & 2) ? -a : a, (q & 2) ? -b : b);
}

// z * w with two fused multiply-adds per component
__device__ __forceinline__ double2 c_mul_fma(double2 z, double2 w) {
    return make_double2(fma(z.x, w.x, -z.y * w.y), fma(z.x, w.y, z.y * w.x));
}

// DPP move of a double / complex within each quad of lanes (quad_perm control;
// also the row controls: 0x141 row_half_mirror, 0x128 row_ror 8)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, CTRL, 0xf, 0xf, false),
                            __builtin_amdgcn_mov_dpp(lo, CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double2 dpp_c(double2 v) { return make_double2(dpp_d<CTRL>(v.x), dpp_d<CTRL>(v.y)); }
static constexpr int QP_XOR1 = 0xb1;    // quad_perm [1, 0, 3, 2]
static constexpr int QP_XOR2 = 0x4e;    // quad_perm [2, 3, 0, 1]
static constexpr int QP_PREV = 0x4b;    // quad_perm [3, 2, 0, 1]: the lane holding the previous time quarter

static constexpr int JCH_MAX = 16;

// a double from the neighbouring lane of the pair (DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ double dpp_d_xor1(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, 0xb1, 0xf, 0xf, false),
                            __builtin_amdgcn_mov_dpp(lo, 0xb1, 0xf, 0xf, false));
}
// RPW realisations per wave (LPR = 64 / RPW lanes each): with N = 540 two
// realisations of 32 chunks of 17 samples keep every lane busy with twice the
// chunk length of one realisation per wave (the per-chunk cis is amortised over
// 17 samples instead of 9).
// PS lanes per chunk split the paths (PS = 2: lane pair, sums joined by a lane
// exchange): long chunks amortise the per-chunk cis without idling lanes.
template <int JCH, int RPW, int PS = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
k_jakes(ChannelK ch, uint64_t seed, uint64_t rep0, int R, double2* __restrict__ ir, const int* __restrict__ chunk_n0,
        int nchunk) {
    extern __shared__ double sm[];
    constexpr int LPR = WAVE / RPW;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = RPW == 1 ? 0 : lane / LPR, sl = RPW == 1 ? lane : lane % LPR;
    const int P = ch.paths;
    double* ds = sm + (size_t)(wv * RPW + sub) * 4 * P;
    double* ph = ds + P;
    double* wr = ph + P;
    double* wi = wr + P;
    const int tap = blockIdx.z;
    const int rl = (blockIdx.y * 4 + wv) * RPW + sub;
    const uint64_t rep = rep0 + (uint64_t)rl;
    for (int p = sl; p < P; p += LPR) {
        const uint32_t e = (uint32_t)(tap + ch.ntap * p);       // rand([Ntap 1 Paths]) column-major
        const uint4 wt = stream_block(seed, rep, STREAM_THETA, 0, e >> 1);
        const uint4 wp = stream_block(seed, rep, STREAM_PHI, 0, e >> 1);
        const double th = (e & 1) ? u53(wt.z, wt.w) : u53(wt.x, wt.y);
        const double phi = (e & 1) ? u53(wp.z, wp.w) : u53(wp.x, wp.y);
        const double d = (ch.model == 0) ? cos((th * 2.0) * M_PI) * ch.fD : (2.0 * (th - 0.5)) * ch.fD;
        double sn, cs;
        sincos(TWO_PI * (d * ch.dt), &sn, &cs);
        ds[p] = d;
        ph[p] = phi;
        wr[p] = cs;
        wi[p] = sn;
    }
    __syncthreads();
    // chunk_n0: the first samples of the chunks to form (the samples some Q^H
    // row reads, JakesChunks); otherwise all N samples in consecutive chunks
    const int ck = blockIdx.x * (LPR / PS) + sl / PS, par = sl % PS;
    if (chunk_n0 && ck >= nchunk) return;
    const int n0 = chunk_n0 ? chunk_n0[ck] : ck * JCH;
    if (n0 >= ch.N) return;
    const double t0 = (double)n0 * ch.dt;
    double2 acc[JCH];
#pragma unroll
    for (int i = 0; i < JCH; ++i) acc[i] = make_double2(0.0, 0.0);
    // Per path and chunk: one exact cis at the chunk start, one rotation for the
    // second sample, then the three-term recurrence z[i+1] = 2 cos(theta) z[i] -
    // z[i-1] (two FMAs per sample instead of a complex rotation's four; its
    // rounding error grows at most like i^2 eps, ~1e-14 at 16 samples).  Four
    // paths per step: four independent recurrences interleave (two left the
    // wave waiting on FMA latency half its cycles, SQ_WAIT_INST_ANY 0.53), and
    // the accumulation costs 1.5 adds per path and sample instead of 2.  With
    // 24-sample chunks (PS = 2) two paths per step (4 need 204 VGPRs); pinned
    // to 3 waves / SIMD (154 VGPRs, no spill since the lane pair exchanges
    // half-chunks below; unpinned the compiler took 204 and 2 waves: 2.04 ->
    // 1.90 ms per step at C2; 4 waves spill inside the path loop: 1.97 ms).
    constexpr int PU = PS == 2 ? 2 : 4;
    const int pend = (par + 1) * P / PS;
    int p = par * P / PS;
    for (; p + PU - 1 < pend; p += PU) {
        double2 a[PU], b[PU];
        double c[PU];
#pragma unroll
        for (int j = 0; j < PU; ++j) {
            a[j] = cis_turns(ph[p + j] + ds[p + j] * t0);
            c[j] = 2.0 * wr[p + j];
            b[j] = c_mul_fma(a[j], make_double2(wr[p + j], wi[p + j]));
        }
        acc[0].x += PU == 4 ? (a[0].x + a[1].x) + (a[2 % PU].x + a[3 % PU].x) : a[0].x + a[1].x;
        acc[0].y += PU == 4 ? (a[0].y + a[1].y) + (a[2 % PU].y + a[3 % PU].y) : a[0].y + a[1].y;
#pragma unroll
        for (int i = 1; i < JCH; ++i) {
            acc[i].x += PU == 4 ? (b[0].x + b[1].x) + (b[2 % PU].x + b[3 % PU].x) : b[0].x + b[1].x;
            acc[i].y += PU == 4 ? (b[0].y + b[1].y) + (b[2 % PU].y + b[3 % PU].y) : b[0].y + b[1].y;
            if (i + 1 < JCH) {
#pragma unroll
                for (int j = 0; j < PU; ++j) {
                    const double2 n = make_double2(fma(c[j], b[j].x, -a[j].x), fma(c[j], b[j].y, -a[j].y));
                    a[j] = b[j];
                    b[j] = n;
                }
            }
        }
    }
    for (; p < pend; ++p) {
        double2 a = cis_turns(ph[p] + ds[p] * t0);
        const double2 w = make_double2(wr[p], wi[p]);
        const double c = 2.0 * wr[p];
        double2 b = c_mul_fma(a, w);
        acc[0].x += a.x;
        acc[0].y += a.y;
#pragma unroll
        for (int i = 1; i < JCH; ++i) {
            acc[i].x += b.x;
            acc[i].y += b.y;
            if (i + 1 < JCH) {
                const double2 n = make_double2(fma(c, b.x, -a.x), fma(c, b.y, -a.y));
                a = b;
                b = n;
            }
        }
    }
    const double sp = sqrt((double)P);
    const double g = ch.sqrt_pdp[tap];
    if constexpr (PS == 2) {
        // the lane pair's path sums: each lane keeps the half of the chunk it
        // stores and receives the partner's partial sums of that half (one
        // exchange per sample instead of two; a + b == b + a, same sums)
        constexpr int H = JCH / 2;
#pragma unroll
        for (int k = 0; k < H; ++k) {
            const double sx = par ? acc[k].x : acc[k + H].x, sy = par ? acc[k].y : acc[k + H].y;
            const double ox = par ? acc[k + H].x : acc[k].x, oy = par ? acc[k + H].y : acc[k].y;
            const double vx = ox + __shfl_xor(sx, 1), vy = oy + __shfl_xor(sy, 1);
            const int n = n0 + k + H * par;
            if (n < ch.N) ir[((size_t)tap * ch.N + n) * R + rl] = make_double2(g * (vx / sp), g * (vy / sp));
        }
    } else {
#pragma unroll
        for (int i = 0; i < JCH; ++i) {
            const int n = n0 + i;
            if (n < ch.N) ir[((size_t)tap * ch.N + n) * R + rl] = make_double2(g * (acc[i].x / sp), g * (acc[i].y / sp));
        }
    }
}

template <int JCH, int RPW = 1, int PS = 1>
static void launch_jakes_t(hipStream_t s, const ChannelK& ch, uint64_t seed, uint64_t rep0, int R, double2* ir,
                           const int* chunk_n0 = nullptr, int nck = 0) {
    constexpr int CPW = WAVE / RPW / PS;          // chunks per realisation and wave
    const int nchunk = chunk_n0 ? nck : (ch.N + JCH - 1) / JCH;
    dim3 grid((nchunk + CPW - 1) / CPW, R / (4 * RPW), ch.ntap);
    hipLaunchKernelGGL((k_jakes<JCH, RPW, PS>), grid, dim3(256), (size_t)4 * RPW * 4 * ch.paths * sizeof(double), s, ch,
                       seed, rep0, R, ir, chunk_n0, nchunk);
}

// The same sum of sinusoids over a 24-sample chunk by phase moments (r03):
// with theta_p = 2 pi fD_p dt (radians per sample), the chunk centre c and
// z_p = exp(j 2 pi (phi_p + fD_p c dt)),
//   sum_p exp(j 2 pi (phi_p + fD_p (c + k) dt)) = sum_p z_p exp(j theta_p k)
//     = sum_m M_m (j k)^m / m!,   M_m = sum_p z_p theta_p^m,   |k| <= 11.5,
// exact up to the Taylor remainder sum_p |theta_p k|^(MT+1) / (MT+1)!: the
// launcher uses it only while |theta| 11.5 <= 0.3 (C2: 0.233; remainder
// < 1e-14 at 200 paths, far inside the 1e-12 parity tolerance of the IR).  Per
// path and chunk one cis and MT (multiply + 2 FMAs) instead of the recurrence's
// 24 x (2 FMAs + accumulation); the moments of the lane pair's two path halves
// are summed by one exchange, then each lane evaluates its 12 samples by Horner
// (2 FMAs per term).  ~1.8x fewer instructions than k_jakes on the same chunks.
template <int RPW, int MT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
k_jakes_mom(ChannelK ch, uint64_t seed, uint64_t rep0, int R, double2* __restrict__ ir, const int* __restrict__ chunk_n0,
            int nchunk) {
    constexpr int JCH = 24, H = JCH / 2, PS = 2;
    extern __shared__ double sm[];
    constexpr int LPR = WAVE / RPW;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = RPW == 1 ? 0 : lane / LPR, sl = RPW == 1 ? lane : lane % LPR;
    const int P = ch.paths;
    double* ds = sm + (size_t)(wv * RPW + sub) * 3 * P;
    double* ph = ds + P;
    double* th = ph + P;
    const int tap = blockIdx.z;
    const int rl = (blockIdx.y * 4 + wv) * RPW + sub;
    const uint64_t rep = rep0 + (uint64_t)rl;
    for (int p = sl; p < P; p += LPR) {
        const uint32_t e = (uint32_t)(tap + ch.ntap * p);       // rand([Ntap 1 Paths]) column-major
        const uint4 wt = stream_block(seed, rep, STREAM_THETA, 0, e >> 1);
        const uint4 wp = stream_block(seed, rep, STREAM_PHI, 0, e >> 1);
        const double t = (e & 1) ? u53(wt.z, wt.w) : u53(wt.x, wt.y);
        const double phi = (e & 1) ? u53(wp.z, wp.w) : u53(wp.x, wp.y);
        const double d = (ch.model == 0) ? cos((t * 2.0) * M_PI) * ch.fD : (2.0 * (t - 0.5)) * ch.fD;
        ds[p] = d;
        ph[p] = phi;
        th[p] = TWO_PI * (d * ch.dt);
    }
    __syncthreads();
    const int ck = blockIdx.x * (LPR / PS) + sl / PS, par = sl % PS;
    if (ck >= nchunk) return;
    const int n0 = chunk_n0[ck];
    if (n0 >= ch.N) return;
    const double tc = ((double)n0 + 0.5 * (JCH - 1)) * ch.dt;
    double2 M[MT + 1];
#pragma unroll
    for (int m = 0; m <= MT; ++m) M[m] = make_double2(0.0, 0.0);
    const int pend = (par + 1) * P / PS;
    int p = par * P / PS;
    for (; p + 1 < pend; p += 2) {
        const double2 z0 = cis_turns(ph[p] + ds[p] * tc), z1 = cis_turns(ph[p + 1] + ds[p + 1] * tc);
        const double t0 = th[p], t1 = th[p + 1];
        M[0].x += z0.x + z1.x;
        M[0].y += z0.y + z1.y;
        double w0 = 1.0, w1 = 1.0;
#pragma unroll
        for (int m = 1; m <= MT; ++m) {
            w0 *= t0;
            w1 *= t1;
            M[m].x = fma(z1.x, w1, fma(z0.x, w0, M[m].x));
            M[m].y = fma(z1.y, w1, fma(z0.y, w0, M[m].y));
        }
    }
    if (p < pend) {
        const double2 z0 = cis_turns(ph[p] + ds[p] * tc);
        const double t0 = th[p];
        M[0].x += z0.x;
        M[0].y += z0.y;
        double w0 = 1.0;
#pragma unroll
        for (int m = 1; m <= MT; ++m) {
            w0 *= t0;
            M[m].x = fma(z0.x, w0, M[m].x);
            M[m].y = fma(z0.y, w0, M[m].y);
        }
    }
    // the lane pair's moments summed (a + b == b + a: both lanes hold the same total)
#pragma unroll
    for (int m = 0; m <= MT; ++m) {
        M[m].x += dpp_d_xor1(M[m].x);
        M[m].y += dpp_d_xor1(M[m].y);
    }
    const double gs = ch.sqrt_pdp[tap] / sqrt((double)P);
    // M_m / m! (compile-time reciprocals): Horner then takes two FMAs per term
    // (a kp / (m + 1) per term compiles to an IEEE division sequence: 1.27 ->
    // 1.15 ms per 65536 realisations at C2)
    {
        double f = 1.0;
#pragma unroll
        for (int m = 2; m <= MT; ++m) {
            f /= (double)m;                                     // constant-folded
            M[m].x *= f;
            M[m].y *= f;
        }
    }
#pragma unroll
    for (int k = 0; k < H; ++k) {
        // sample n0 + kk, offset kk - 11.5 from the centre: Horner in (j kp)
        const int kk = k + H * par;
        const double kp = (double)kk - 0.5 * (JCH - 1);
        double2 acc = M[MT];
#pragma unroll
        for (int m = MT - 1; m >= 0; --m) {
            const double ax = acc.x;
            acc.x = fma(-kp, acc.y, M[m].x);
            acc.y = fma(kp, ax, M[m].y);
        }
        const int n = n0 + kk;
        if (n < ch.N) ir[((size_t)tap * ch.N + n) * R + rl] = make_double2(gs * acc.x, gs * acc.y);
    }
}

// Anchors over groups of chunks (r03, k_jakes_grp): the moment sum of
// k_jakes_mom taken around the centre c of a run of consecutive chunks instead of
// each chunk's own, with MT terms enough for |theta k| <= JAKES_XMAX (3.0) over the
// run (jakes groups: MT = the smallest of 16 / 24 / 28 with x^(MT+1) / (MT+1)! <=
// 1e-17; the terms peak at e^x / sqrt(2 pi x) ~ 5 before they fall, so the
// rounding stays ~ 5 P eps).  At C2 two anchors per realisation and tap replace
// fourteen: per path and anchor one cis and MT (multiply + 2 FMAs), LG lanes per
// anchor split the paths and sum their moments by DPP (quad xor 1 / 2, row half
// mirror, row rotate 8), then split the run's samples for Horner.
template <int MT, int LG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_jakes_grp(ChannelK ch, uint64_t seed, uint64_t rep0, int R,
                                                   double2* __restrict__ ir, const int* __restrict__ chunk_n0,
                                                   const int2* __restrict__ grp, int ngrp) {
    static_assert(LG == 4 || LG == 8 || LG == 16, "lanes per anchor");
    constexpr int JCH = JakesChunks::LEN, RPW = 2, LPR = WAVE / RPW, GPB = LPR / LG;
    extern __shared__ double sm[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = lane / LPR, sl = lane % LPR;
    const int P = ch.paths;
    double* ds = sm + (size_t)(wv * RPW + sub) * 3 * P;
    double* ph = ds + P;
    double* th = ph + P;
    const int tap = blockIdx.z;
    const int rl = (blockIdx.y * 4 + wv) * RPW + sub;
    const uint64_t rep = rep0 + (uint64_t)rl;
    for (int p = sl; p < P; p += LPR) {
        const uint32_t e = (uint32_t)(tap + ch.ntap * p);       // rand([Ntap 1 Paths]) column-major
        const uint4 wt = stream_block(seed, rep, STREAM_THETA, 0, e >> 1);
        const uint4 wp = stream_block(seed, rep, STREAM_PHI, 0, e >> 1);
        const double t = (e & 1) ? u53(wt.z, wt.w) : u53(wt.x, wt.y);
        const double phi = (e & 1) ? u53(wp.z, wp.w) : u53(wp.x, wp.y);
        const double d = (ch.model == 0) ? cos((t * 2.0) * M_PI) * ch.fD : (2.0 * (t - 0.5)) * ch.fD;
        ds[p] = d;
        ph[p] = phi;
        th[p] = TWO_PI * (d * ch.dt);
    }
    __syncthreads();
    const int gi = blockIdx.x * GPB + sl / LG, li = sl % LG;
    if (gi >= ngrp) return;                                     // whole groups leave together
    const int2 gr = grp[gi];
    const int na = chunk_n0[gr.x], nb = chunk_n0[gr.x + gr.y - 1];
    const double cen = 0.5 * ((double)na + (double)nb + (JCH - 1));
    const double tc = cen * ch.dt;
    double2 M[MT + 1];
#pragma unroll
    for (int m = 0; m <= MT; ++m) M[m] = make_double2(0.0, 0.0);
    int p = li;
    for (; p + LG < P; p += 2 * LG) {
        const double2 z0 = cis_turns(ph[p] + ds[p] * tc), z1 = cis_turns(ph[p + LG] + ds[p + LG] * tc);
        const double t0 = th[p], t1 = th[p + LG];
        M[0].x += z0.x + z1.x;
        M[0].y += z0.y + z1.y;
        double w0 = 1.0, w1 = 1.0;
#pragma unroll
        for (int m = 1; m <= MT; ++m) {
            w0 *= t0;
            w1 *= t1;
            M[m].x = fma(z1.x, w1, fma(z0.x, w0, M[m].x));
            M[m].y = fma(z1.y, w1, fma(z0.y, w0, M[m].y));
        }
    }
    if (p < P) {
        const double2 z0 = cis_turns(ph[p] + ds[p] * tc);
        const double t0 = th[p];
        M[0].x += z0.x;
        M[0].y += z0.y;
        double w0 = 1.0;
#pragma unroll
        for (int m = 1; m <= MT; ++m) {
            w0 *= t0;
            M[m].x = fma(z0.x, w0, M[m].x);
            M[m].y = fma(z0.y, w0, M[m].y);
        }
    }
    // the group's moments summed into every lane of the group; then M_m / m!
    double f = 1.0;
#pragma unroll
    for (int m = 0; m <= MT; ++m) {
        double mx = M[m].x, my = M[m].y;
        mx += dpp_d<QP_XOR1>(mx);
        my += dpp_d<QP_XOR1>(my);
        mx += dpp_d<QP_XOR2>(mx);
        my += dpp_d<QP_XOR2>(my);
        if constexpr (LG >= 8) {
            mx += dpp_d<0x141>(mx);                             // row_half_mirror: the other quad of 8
            my += dpp_d<0x141>(my);
        }
        if constexpr (LG >= 16) {
            mx += dpp_d<0x128>(mx);                             // row_ror 8: the other half of the row
            my += dpp_d<0x128>(my);
        }
        if (m >= 2) f /= (double)m;                             // constant-folded
        M[m] = make_double2(mx * f, my * f);
    }
    const double gs = ch.sqrt_pdp[tap] / sqrt((double)P);
    const int ns = gr.y * JCH;
    for (int j = li; j < ns; j += LG) {
        const int n = chunk_n0[gr.x + j / JCH] + j % JCH;
        const double kp = (double)n - cen;
        double2 acc = M[MT];
#pragma unroll
        for (int m = MT - 1; m >= 0; --m) {
            const double ax = acc.x;
            acc.x = fma(-kp, acc.y, M[m].x);
            acc.y = fma(kp, ax, M[m].y);
        }
        if (n < ch.N) ir[((size_t)tap * ch.N + n) * R + rl] = make_double2(gs * acc.x, gs * acc.y);
    }
}

// k_jakes_grp for channels with two non-zero taps (r06; C2-C4's VehicularA at
// 360 kHz): a wave holds 2 realisations x 2 taps x NG anchor groups of LG =
// 16 / NG lanes.  One Philox block of the THETA / PHI streams carries path p's
// uniforms of BOTH taps (element e = tap + 2 p, counter e >> 1 = p: words (x, y)
// for tap 0, (z, w) for tap 1), so each block is drawn once instead of once per
// tap (k_jakes_grp's grid is per tap), and the four (realisation, tap) pairs of
// a wave split its lanes four ways: an anchor's moments sum over LG = 8 lanes at
// C2 (three DPP stages instead of four).  LDS: [wave][realisation][tap]{d, phi}
// per path; theta = 2 pi d dt is formed where it is used (the same expression
// as k_jakes_grp's table).  Same moments, anchors and Horner evaluation.
template <int MT, int LG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_jakes_grp2(ChannelK ch, uint64_t seed, uint64_t rep0, int R, double2* __restrict__ ir,
             const int* __restrict__ chunk_n0, const int2* __restrict__ grp, int ngrp) {
    static_assert(LG == 4 || LG == 8 || LG == 16, "lanes per anchor");
    constexpr int JCH = JakesChunks::LEN, RPW = 2, NG = 16 / LG;
    extern __shared__ double sm[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int P = ch.paths;
    double* wbase = sm + (size_t)wv * RPW * 4 * P;              // [sub][tap][d | phi][P]
    {
        const int sub = lane >> 5, sl = lane & 31;
        const uint64_t rep = rep0 + (uint64_t)((blockIdx.x * 4 + wv) * RPW + sub);
        double* d = wbase + (size_t)sub * 4 * P;
        for (int p = sl; p < P; p += 32) {
            const uint4 wt = stream_block(seed, rep, STREAM_THETA, 0, (uint32_t)p);
            const uint4 wp = stream_block(seed, rep, STREAM_PHI, 0, (uint32_t)p);
            const double t0 = u53(wt.x, wt.y), t1 = u53(wt.z, wt.w);
            d[p] = (ch.model == 0) ? cos((t0 * 2.0) * M_PI) * ch.fD : (2.0 * (t0 - 0.5)) * ch.fD;
            d[P + p] = u53(wp.x, wp.y);
            d[2 * P + p] = (ch.model == 0) ? cos((t1 * 2.0) * M_PI) * ch.fD : (2.0 * (t1 - 0.5)) * ch.fD;
            d[3 * P + p] = u53(wp.z, wp.w);
        }
    }
    __syncthreads();
    // lane -> (realisation sub, tap, anchor group gi), LG lanes per anchor
    const int g = lane / LG, li = lane % LG;
    const int sub = g / (2 * NG), tap = (g / NG) & 1, gi = g % NG;
    if (gi >= ngrp) return;
    const double* ds = wbase + (size_t)sub * 4 * P + (size_t)tap * 2 * P;
    const double* ph = ds + P;
    const int rl = (blockIdx.x * 4 + wv) * RPW + sub;
    const int2 gr = grp[gi];
    const int na = chunk_n0[gr.x], nb = chunk_n0[gr.x + gr.y - 1];
    const double cen = 0.5 * ((double)na + (double)nb + (JCH - 1));
    const double tc = cen * ch.dt;
    double2 M[MT + 1];
#pragma unroll
    for (int m = 0; m <= MT; ++m) M[m] = make_double2(0.0, 0.0);
    int p = li;
    for (; p + LG < P; p += 2 * LG) {
        const double d0 = ds[p], d1 = ds[p + LG];
        const double2 z0 = cis_turns(ph[p] + d0 * tc), z1 = cis_turns(ph[p + LG] + d1 * tc);
        const double t0 = TWO_PI * (d0 * ch.dt), t1 = TWO_PI * (d1 * ch.dt);
        M[0].x += z0.x + z1.x;
        M[0].y += z0.y + z1.y;
        double w0 = 1.0, w1 = 1.0;
#pragma unroll
        for (int m = 1; m <= MT; ++m) {
            w0 *= t0;
            w1 *= t1;
            M[m].x = fma(z1.x, w1, fma(z0.x, w0, M[m].x));
            M[m].y = fma(z1.y, w1, fma(z0.y, w0, M[m].y));
        }
    }
    if (p < P) {
        const double d0 = ds[p];
        const double2 z0 = cis_turns(ph[p] + d0 * tc);
        const double t0 = TWO_PI * (d0 * ch.dt);
        M[0].x += z0.x;
        M[0].y += z0.y;
        double w0 = 1.0;
#pragma unroll
        for (int m = 1; m <= MT; ++m) {
            w0 *= t0;
            M[m].x = fma(z0.x, w0, M[m].x);
            M[m].y = fma(z0.y, w0, M[m].y);
        }
    }
    double f = 1.0;
#pragma unroll
    for (int m = 0; m <= MT; ++m) {
        double mx = M[m].x, my = M[m].y;
        mx += dpp_d<QP_XOR1>(mx);
        my += dpp_d<QP_XOR1>(my);
        mx += dpp_d<QP_XOR2>(mx);
        my += dpp_d<QP_XOR2>(my);
        if constexpr (LG >= 8) {
            mx += dpp_d<0x141>(mx);                             // row_half_mirror: the other quad of 8
            my += dpp_d<0x141>(my);
        }
        if constexpr (LG >= 16) {
            mx += dpp_d<0x128>(mx);                             // row_ror 8: the other half of the row
            my += dpp_d<0x128>(my);
        }
        if (m >= 2) f /= (double)m;                             // constant-folded
        M[m] = make_double2(mx * f, my * f);
    }
    const double gs = ch.sqrt_pdp[tap] / sqrt((double)P);
    const int ns = gr.y * JCH;
    for (int j = li; j < ns; j += LG) {
        const int n = chunk_n0[gr.x + j / JCH] + j % JCH;
        const double kp = (double)n - cen;
        double2 acc = M[MT];
#pragma unroll
        for (int m = MT - 1; m >= 0; --m) {
            const double ax = acc.x;
            acc.x = fma(-kp, acc.y, M[m].x);
            acc.y = fma(kp, ax, M[m].y);
        }
        if (n < ch.N) ir[((size_t)tap * ch.N + n) * R + rl] = make_double2(gs * acc.x, gs * acc.y);
    }
}

// Box-Muller pair of the random-stream spec (include/dsce.h): u1 = u53(w0,w1),
// u2 = u53(w2,w3), (re, im) = sqrt(-2 log(1-u1)) (cos, sin)(2 pi u2).
//
// r05: table-driven, ~48 FP64 instructions per pair instead of
// ~118 (the library log alone was 68, a double-double evaluation: 43 v_add_f64).
// Same spec, same uniforms; the pair differs from the NumPy oracle's
// np.log / np.sqrt / np.cos / np.sin evaluation by a few units in the last
// place (tests/test_bm_tables.py restates the algorithm and bounds it;
// test_gpu_doubly_flat.py::test_device_normals_match_oracle on the box).
// Tables: csrc/bm_tables.h (tools/gen_bm_tables.py).
//
// x = 1 - u1 exactly (a multiple of 2^-53 in (0, 1], built by two exact FMAs
// from the 27 + 26 bits), always a normal double.
__device__ __forceinline__ double one_minus_u53(uint32_t a, uint32_t b) {
    return fma(-(double)(a >> 5), 0x1p-27, fma(-(double)(b >> 6), 0x1p-53, 1.0));
}

// -2 log x for x in (0, 1]: x = m 2^(E - 1022), m in [1/2, 1) taken from the bit
// pattern (three integer ops, no frexp); interval i = top 7 bits of m with
// lt[i] = (invc, 2 log invc); r = m invc - 1, |r| <= 2^-7 (2^-8 except at the
// interval of m = 1/2); -2 log1p(r) = -2 r + r^2 P(r) with the Taylor terms to
// r^7 (truncation < 2e-18).  For x in [1/2, 1) there is no ln 2 term, so the
// result's only rounding is the table value's (of the result's size); x -> 1
// lands in the interval whose centre is 1 (invc = 1, table value 0): full
// relative precision; x = 1 (E - 1022 = 1, invc = 2) gives exactly 0.
__device__ __forceinline__ double m2log_unit(double x, const double2* __restrict__ lt) {
    const int hi = __double2hiint(x);
    const double m = __hiloint2double((hi & 0x000FFFFF) | 0x3FE00000, __double2loint(x));
    const double2 t = lt[(hi >> 13) & 127];
    const double ed = (double)((hi >> 20) - 1022);           // E - 1022 (x > 0: no sign bit)
    const double r = fma(m, t.x, -1.0);
    double p = -2.0 / 7.0;
    p = fma(p, r, 1.0 / 3.0);
    p = fma(p, r, -2.0 / 5.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, -2.0 / 3.0);
    p = fma(p, r, 1.0);
    const double s1 = fma(ed, -1.3862943611198906, t.y);      // -2 ln 2
    return s1 + fma(r, -2.0, (r * r) * p);
}

// sqrt(a) for 0 <= a < 2^1000 (a = 0 -> ~1e-150): v_rsq_f64 and the Newton
// steps of the library sqrt without its range scaling (a is never denormal)
__device__ __forceinline__ double sqrt_bm(double a) {
    a = fmax(a, 1e-300);
    const double y = __builtin_amdgcn_rsq(a);
    double g = a * y, h = 0.5 * y;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    double d = fma(-g, g, a);
    g = fma(d, h, g);
    d = fma(-g, g, a);
    return fma(d, h, g);
}

// (cos, sin)(2 pi u2), u2 = u53(a, b): interval j = top 8 bits of u2, ct[j] =
// cis(2 pi (j + 1/2) / 256), theta = 2 pi (u2 - (j + 1/2) / 256) in
// [-pi/256, pi/256) from the remaining 19 + 26 bits; sin to theta^5, cos - 1 to
// theta^6 (truncation < 1e-17), then ct[j] (1 + (cos - 1) + i sin).
__device__ __forceinline__ double2 cis_u53(uint32_t a, uint32_t b, const double2* __restrict__ ct) {
    const double2 t = ct[a >> 24];
    const double th = fma((double)((a >> 5) & 0x7FFFFu), 0x1p-27 * 6.283185307179586,
                          fma((double)(b >> 6), 0x1p-53 * 6.283185307179586, -0.012271846303085130));
    const double t2 = th * th;
    const double s = fma(th * t2, fma(t2, 1.0 / 120.0, -1.0 / 6.0), th);
    const double cm1 = t2 * fma(fma(t2, -1.0 / 720.0, 1.0 / 24.0), t2, -0.5);
    return make_double2(fma(t.x, cm1, fma(-t.y, s, t.x)), fma(t.y, cm1, fma(t.x, s, t.y)));
}

// The pair's radius and angle; lt / ct: the tables (LDS copies in k_txrx_fft,
// the __constant__ originals elsewhere: the same values, the same draws).
__device__ __forceinline__ void bm_parts(uint4 w, const double2* __restrict__ lt, const double2* __restrict__ ct,
                                         double& rad, double2& cz) {
    rad = sqrt_bm(m2log_unit(one_minus_u53(w.x, w.y), lt));
    cz = cis_u53(w.z, w.w, ct);
}

__device__ __forceinline__ double2 normal_pair(uint4 w, const double2* __restrict__ lt = kLogT,
                                               const double2* __restrict__ ct = kCisT) {
    double rad;
    double2 cz;
    bm_parts(w, lt, ct, rad, cz);
    return make_double2(rad * cz.x, rad * cz.y);
}

// r0 + sc z of one noise sample (every AWGN path: k_noise, LoadNoisy,
// k_txrx_fft — one expression, so the fused and unfused paths draw the same bits)
__device__ __forceinline__ double2 noise_add(double2 r0, double sc, uint4 w, const double2* __restrict__ lt = kLogT,
                                             const double2* __restrict__ ct = kCisT) {
    double rad;
    double2 cz;
    bm_parts(w, lt, ct, rad, cz);
    const double rs = sc * rad;
    return make_double2(fma(rs, cz.x, r0.x), fma(rs, cz.y, r0.y));
}

// ---------------------------------------------------------------------------
// a2 (MaximumDopplerShift == 0): time-invariant block fading, FastFading.m:241-246:
// IR[tap] = 1/sqrt(2) sqrt(PDPn[tap]) (randn + j randn), one value per
// realisation that GetConvolutionMatrix repeats over all N samples
// (FastFading.m:288-291).  With the 'Flat' PDP this is the doubly-flat
// h = sqrt(1/2) (randn + j randn) of SimpleVersion_DoublyFlat.m:123.
// RNG: THETA stream, sub 0, counter = non-zero tap index.  grid (R/64,
// ceil(N/64), ntap), lane = realisation.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_static(ChannelK ch, uint64_t seed, uint64_t rep0, int R,
                                               double2* __restrict__ ir) {
    const int rl = blockIdx.x * WAVE + threadIdx.x;
    const int q = blockIdx.z;
    const double2 z = normal_pair(stream_block(seed, rep0 + (uint64_t)rl, STREAM_THETA, 0, (uint32_t)q));
    const double c = (1.0 / sqrt(2.0)) * ch.sqrt_pdp[q];
    const double2 v = make_double2(c * z.x, c * z.y);
    const int n0 = blockIdx.y * 64;
    for (int n = n0; n < n0 + 64 && n < ch.N; ++n) ir[((size_t)q * ch.N + n) * R + rl] = v;
}

// ---------------------------------------------------------------------------
// a2, 'Discrete-Jakes' / 'Discrete-Uniform' (FastFading.m:203-221): the IFFT of
// [sqrt(S(nd+1:end)) .* G1; zeros; sqrt(S(1:nd)) .* G2] with
// G = N/sqrt(2) (randn + j randn) sqrt(PDPn) has only the 2 nd + 1 Doppler bins
// f = -nd..nd non-zero, so it is evaluated directly:
//   IR[n, tap] = sum_f c_f exp(j 2 pi f n / N),
//   c_f = sqrt(S_f) sqrt(PDPn[tap]) / sqrt(2) (re_f + j im_f)
// (the ifft's 1/N cancels the N of G).  RNG: THETA stream, sub 1, counter
// (f + nd) + (2 nd + 1) tap, Box-Muller pair.  Lane = realisation, DCH samples
// per lane: exact phase (f n mod N in integers) at the chunk start, then
// rotations.  grid (R/64, ceil(N/DCH), ntap).
// ---------------------------------------------------------------------------
static constexpr int DCH = 16;
__global__ void __launch_bounds__(64) k_discrete(ChannelK ch, uint64_t seed, uint64_t rep0, int R,
                                                 double2* __restrict__ ir) {
    const int rl = blockIdx.x * WAVE + threadIdx.x;
    const int q = blockIdx.z;
    const uint64_t rep = rep0 + (uint64_t)rl;
    const int n0 = blockIdx.y * DCH;
    const int nb = 2 * ch.nd + 1;
    double2 acc[DCH];
#pragma unroll
    for (int i = 0; i < DCH; ++i) acc[i] = make_double2(0.0, 0.0);
    const double g = ch.sqrt_pdp[q] / sqrt(2.0);
    for (int b = 0; b < nb; ++b) {
        const int f = b - ch.nd;
        const double2 z0 = normal_pair(stream_block(seed, rep, STREAM_THETA, 1, (uint32_t)(b + nb * q)));
        const double a = ch.sqrt_dspec[b] * g;
        const double2 cf = make_double2(a * z0.x, a * z0.y);
        const long long m = (((long long)f * n0) % ch.N + ch.N) % ch.N;
        double2 z = c_mul(cf, cis_turns((double)m / (double)ch.N));
        const double2 w = cis_turns((double)f / (double)ch.N);
#pragma unroll
        for (int i = 0; i < DCH; ++i) {
            acc[i].x += z.x;
            acc[i].y += z.y;
            if (i + 1 < DCH) z = c_mul_fma(z, w);
        }
    }
#pragma unroll
    for (int i = 0; i < DCH; ++i) {
        const int n = n0 + i;
        if (n < ch.N) ir[((size_t)q * ch.N + n) * R + rl] = acc[i];
    }
}

int launch_jakes(hipStream_t s, const Opts& op, const ChannelK& ch, uint64_t seed, uint64_t rep0, int R,
                  double2* ir, const JakesChunks* jc) {
    if (ch.fD == 0.0) {
        hipLaunchKernelGGL(k_static, dim3(R / WAVE, (ch.N + 63) / 64, ch.ntap), dim3(WAVE), 0, s, ch, seed, rep0, R, ir);
        return JAKES_KIND_OTHER;
    }
    if (ch.model >= 2) {
        hipLaunchKernelGGL(k_discrete, dim3(R / WAVE, (ch.N + DCH - 1) / DCH, ch.ntap), dim3(WAVE), 0, s, ch, seed,
                           rep0, R, ir);
        return JAKES_KIND_OTHER;
    }
    // only the samples some Q^H row reads (OFDM: the FFT windows): chunks of 24
    // aligned to them, two realisations per wave, a lane pair per chunk
    // splitting the paths (12-sample chunks, one lane each: 2.37 ms per
    // 65536 realisations at C2, the per-chunk cis ~45 % of the instructions)
    if (jc && jc->n0 && op.jakes_win && R % 8 == 0 && (size_t)8 * 4 * ch.paths * sizeof(double) <= 64 * 1024) {
        // the phase-moment form where its Taylor remainder is negligible
        // (|theta| (LEN - 1) / 2 <= 0.3), else the recurrence
        // two non-zero taps and 1 / 2 / 4 anchor groups: both taps in one wave
        // (k_jakes_grp2: each Philox block drawn once, LG = 16 / groups)
        if (op.jakes_mom == 2 && jc->ngrp > 0 && op.jakes_grp2 && ch.ntap == 2 &&
            (jc->ngrp == 1 || jc->ngrp == 2 || jc->ngrp == 4) && (size_t)32 * ch.paths * sizeof(double) <= 64 * 1024) {
            const dim3 grid(R / 8);
            const size_t lds = (size_t)32 * ch.paths * sizeof(double);
#define LAUNCH_JGRP2(MT_, NG_)                                                                                 \
    if (jc->mt == MT_ && jc->ngrp == NG_) {                                                                   \
        hipLaunchKernelGGL((k_jakes_grp2<MT_, 16 / NG_>), grid, dim3(256), lds, s, ch, seed, rep0, R, ir,     \
                           jc->n0, jc->grp, jc->ngrp);                                                        \
        return JAKES_KIND_GRP;                                                                                \
    }
            LAUNCH_JGRP2(16, 1) LAUNCH_JGRP2(16, 2) LAUNCH_JGRP2(16, 4)
            LAUNCH_JGRP2(24, 1) LAUNCH_JGRP2(24, 2) LAUNCH_JGRP2(24, 4)
            LAUNCH_JGRP2(28, 1) LAUNCH_JGRP2(28, 2) LAUNCH_JGRP2(28, 4)
#undef LAUNCH_JGRP2
        }
        if (op.jakes_mom == 2 && jc->ngrp > 0) {
            constexpr int RPW = 2;
            const int gpb = WAVE / RPW / jc->lg;
            dim3 grid((jc->ngrp + gpb - 1) / gpb, R / (4 * RPW), ch.ntap);
            const size_t lds = (size_t)4 * RPW * 3 * ch.paths * sizeof(double);
#define LAUNCH_JGRP(MT_, LG_)                                                                                 \
    if (jc->mt == MT_ && jc->lg == LG_) {                                                                    \
        hipLaunchKernelGGL((k_jakes_grp<MT_, LG_>), grid, dim3(256), lds, s, ch, seed, rep0, R, ir, jc->n0,  \
                           jc->grp, jc->ngrp);                                                               \
        return JAKES_KIND_GRP;                                                                               \
    }
            LAUNCH_JGRP(16, 4) LAUNCH_JGRP(16, 8) LAUNCH_JGRP(16, 16)
            LAUNCH_JGRP(24, 4) LAUNCH_JGRP(24, 8) LAUNCH_JGRP(24, 16)
            LAUNCH_JGRP(28, 4) LAUNCH_JGRP(28, 8) LAUNCH_JGRP(28, 16)
#undef LAUNCH_JGRP
        }
        if (op.jakes_mom && JakesChunks::LEN == 24 && TWO_PI * fabs(ch.fD) * ch.dt * 11.5 <= 0.3) {
            constexpr int RPW = 2, CPW = WAVE / RPW / 2;
            dim3 grid((jc->n + CPW - 1) / CPW, R / (4 * RPW), ch.ntap);
            hipLaunchKernelGGL((k_jakes_mom<RPW, 12>), grid, dim3(256), (size_t)4 * RPW * 3 * ch.paths * sizeof(double),
                               s, ch, seed, rep0, R, ir, jc->n0, jc->n);
            return JAKES_KIND_MOM;
        }
        launch_jakes_t<JakesChunks::LEN, 2, 2>(s, ch, seed, rep0, R, ir, jc->n0, jc->n);
        return JAKES_KIND_OTHER;
    }
    // two realisations per wave (32 lanes each) when that gives chunks of 9-20
    // samples (N 257-640) and R splits into blocks of 8; the LDS path tables
    // then take 64 P bytes per realisation, 51 KB per block at P = 200
    const int jch2 = (ch.N + WAVE / 2 - 1) / (WAVE / 2);
    if (jch2 >= 9 && jch2 <= 20 && R % 8 == 0 && (size_t)8 * 4 * ch.paths * sizeof(double) <= 64 * 1024 &&
        op.jakes_rpw == 2) {
        switch (jch2) {
            case 9: launch_jakes_t<9, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 10: launch_jakes_t<10, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 11: launch_jakes_t<11, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 12: launch_jakes_t<12, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 13: launch_jakes_t<13, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 14: launch_jakes_t<14, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 15: launch_jakes_t<15, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 16: launch_jakes_t<16, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 17: launch_jakes_t<17, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 18: launch_jakes_t<18, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            case 19: launch_jakes_t<19, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
            default: launch_jakes_t<20, 2>(s, ch, seed, rep0, R, ir); return JAKES_KIND_OTHER;
        }
    }
    int jch = (ch.N + WAVE - 1) / WAVE;           // samples per lane: one wave covers N when N <= 1024
    if (jch > JCH_MAX) jch = JCH_MAX;
    switch (jch) {
        case 1: launch_jakes_t<1>(s, ch, seed, rep0, R, ir); break;
        case 2: launch_jakes_t<2>(s, ch, seed, rep0, R, ir); break;
        case 3: launch_jakes_t<3>(s, ch, seed, rep0, R, ir); break;
        case 4: launch_jakes_t<4>(s, ch, seed, rep0, R, ir); break;
        case 5: launch_jakes_t<5>(s, ch, seed, rep0, R, ir); break;
        case 6: launch_jakes_t<6>(s, ch, seed, rep0, R, ir); break;
        case 7: launch_jakes_t<7>(s, ch, seed, rep0, R, ir); break;
        case 8: launch_jakes_t<8>(s, ch, seed, rep0, R, ir); break;
        case 9: launch_jakes_t<9>(s, ch, seed, rep0, R, ir); break;
        case 10: launch_jakes_t<10>(s, ch, seed, rep0, R, ir); break;
        case 11: launch_jakes_t<11>(s, ch, seed, rep0, R, ir); break;
        case 12: launch_jakes_t<12>(s, ch, seed, rep0, R, ir); break;
        case 13: launch_jakes_t<13>(s, ch, seed, rep0, R, ir); break;
        case 14: launch_jakes_t<14>(s, ch, seed, rep0, R, ir); break;
        case 15: launch_jakes_t<15>(s, ch, seed, rep0, R, ir); break;
        default: launch_jakes_t<16>(s, ch, seed, rep0, R, ir); break;
    }
    return JAKES_KIND_OTHER;
}

// ---------------------------------------------------------------------------
// generic banded block matvec: out[row][lane] = sum_k A[row, k] * in(k, lane)
// block 64, 1-D grid of (lanes/64) x nblk blocks.  A's values are wave-uniform
// (scalar loads).  Work order (BandOrder): unit group fastest, or — for passes
// that read per-realisation data shared by the SNR points (the channel taps) —
// SNR point fastest, then row block, then realisation group, each XCD (block b
// runs on XCD b % 8) walking a contiguous range so the reuse stays in one L2.
// ---------------------------------------------------------------------------
struct BandOrder {
    int nug;       // unit groups of 64 lanes
    int nchunk;    // SNR points per unit range (units = snr * R + rep)
    int rgs;       // R / 64
    int xcd;       // 1: SNR-fastest XCD-aware order
};

// Hardware dispatch sends block b to XCD b % 8.  Remap b so that each XCD walks
// one contiguous range of [0, n) — for any n (XCDs x < n % 8 take one block more).
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

__device__ __forceinline__ void band_block(const BandOrder& o, int nblk, int& ug, int& blk, int L, int n) {
    if (o.xcd) {
        L = xcd_remap(L, n);
        const int sn = L % o.nchunk, rest = L / o.nchunk;
        blk = rest % nblk;
        ug = sn * o.rgs + rest / nblk;
    } else {
        ug = L % o.nug;
        blk = L / o.nug;
    }
}
__device__ __forceinline__ void band_block(const BandOrder& o, int nblk, int& ug, int& blk) {
    band_block(o, nblk, ug, blk, blockIdx.x, gridDim.x);
}

template <class In, class Out>
__global__ void __launch_bounds__(64) k_band(Band A, BandOrder ord, In in, Out out) {
    extern __shared__ double2 band_lds[];
    int ug, blk;
    band_block(ord, A.nblk, ug, blk);
    const int lane = ug * WAVE + threadIdx.x;
    Out o = out;
    o.prepare(band_lds);
    const int row0 = A.row0[blk], nrows = A.nrows[blk], klo = A.klo[blk], khi = A.khi[blk];
    const double2* __restrict__ a = A.vals + A.off[blk];
    double2 acc[DSCE_RB];
#pragma unroll
    for (int r = 0; r < DSCE_RB; ++r) acc[r] = make_double2(0.0, 0.0);
    // operands of column k+1 requested before column k's row updates (latency hiding)
    typename In::Regs ld = in.load(klo < khi ? klo : 0, lane);
    for (int k = klo; k < khi; ++k) {
        const typename In::Regs ldn = in.load(k + 1 < khi ? k + 1 : k, lane);
        // keep the scheduler from pulling column k+1's uses up to its loads
        __builtin_amdgcn_sched_barrier(0);
        const double2 x = in.combine(ld);
        const double2* __restrict__ ak = a + (size_t)(k - klo) * DSCE_RB;
#pragma unroll
        for (int r = 0; r < DSCE_RB; ++r) c_fma(acc[r], ak[r], x);
        ld = ldn;
    }
    o.rows(row0, nrows, lane, acc);
    o.finish(lane);
}

template <class In, class Out>
void launch_band(hipStream_t s, const Band& A, int lanes, const BandOrder* ord, const In& in, const Out& out,
                 size_t lds = 0) {
    BandOrder o{lanes / WAVE, 1, 1, 0};
    if (ord) o = *ord;
    hipLaunchKernelGGL((k_band<In, Out>), dim3((lanes / WAVE) * A.nblk), dim3(WAVE), lds, s, A, o, in, out);
}

struct LoadSoA {
    const double2* __restrict__ p;
    int stride;
    typedef double2 Regs;
    __device__ __forceinline__ Regs load(int k, int lane) const { return p[(size_t)k * stride + lane]; }
    __device__ __forceinline__ double2 combine(const Regs& r) const { return r; }
};
// channel taps as the column operand of the diag(D) band: k = n * ntap + tau
struct LoadTapInterleaved {
    const double2* __restrict__ ir;    // [ntap][N][R]
    int N, R, ntap;
    typedef double2 Regs;
    __device__ __forceinline__ Regs load(int k, int lane) const {
        const int n = k / ntap, q = k - n * ntap;
        return ir[((size_t)q * N + n) * R + lane];
    }
    __device__ __forceinline__ double2 combine(const Regs& r) const { return r; }
};
struct StoreSoA {
    double2* __restrict__ p;
    int stride;
    __device__ __forceinline__ void prepare(double2*) {}
    __device__ __forceinline__ void finish(int) {}
    template <int RBN>
    __device__ __forceinline__ void rows(int row0, int nrows, int lane, const double2 (&acc)[RBN]) {
#pragma unroll
        for (int r = 0; r < RBN; ++r)
            if (r < nrows) (*this)(row0 + r, lane, acc[r]);
    }
    __device__ __forceinline__ void operator()(int row, int lane, double2 v) const {
        p[(size_t)row * stride + lane] = v;
    }
};
// (H t)[n] = sum_tau IR[tau][n] t[n - d_tau]  (GetConvolutionMatrix, FastFading.m:284).
// NT > 0: exactly NT taps, unrolled so all 2*NT loads of a column are in flight
// together (load) before the taps are combined; NT == 0: any tap count, loop.
template <int NT>
struct LoadChannelApplied {
    static constexpr int NTS = NT > 0 ? NT : 1;
    const double2* __restrict__ t;     // [N][U]
    const double2* __restrict__ ir;    // [ntap][N][R]
    int U, R, N, ntap;
    int delay[NT > 0 ? NT : DSCE_MAX_TAPS];
    struct Regs {
        double2 a[NTS], b[NTS];
    };
    __device__ __forceinline__ Regs load(int n, int lane) const {
        Regs g;
        const int rep = lane % R;
        if (NT > 0) {
#pragma unroll
            for (int q = 0; q < NTS; ++q) {
                const int m = n - delay[q];
                g.a[q] = ir[((size_t)q * N + n) * R + rep];
                g.b[q] = t[(size_t)(m > 0 ? m : 0) * U + lane];
                if (m < 0) g.b[q] = make_double2(0.0, 0.0);
            }
        } else {
            double2 acc = make_double2(0.0, 0.0);
            for (int q = 0; q < ntap; ++q) {
                const int m = n - delay[q];
                if (m >= 0) c_fma(acc, ir[((size_t)q * N + n) * R + rep], t[(size_t)m * U + lane]);
            }
            g.a[0] = acc;
        }
        return g;
    }
    __device__ __forceinline__ double2 combine(const Regs& g) const {
        if (NT == 0) return g.a[0];
        double2 acc = make_double2(0.0, 0.0);
#pragma unroll
        for (int q = 0; q < NTS; ++q) c_fma(acc, g.a[q], g.b[q]);
        return acc;
    }
};
// y_perf = y - acc + h .* u   (script:541-543 with D - diag(h))
struct StorePerfectIC {
    double2* __restrict__ yperf;
    const double2* __restrict__ y;
    const double2* __restrict__ h;     // [LK][R]
    const double2* __restrict__ u;     // [LK][U]
    int U, R;
    __device__ __forceinline__ void prepare(double2*) {}
    __device__ __forceinline__ void finish(int) {}
    template <int RBN>
    __device__ __forceinline__ void rows(int row0, int nrows, int lane, const double2 (&acc)[RBN]) {
#pragma unroll
        for (int r = 0; r < RBN; ++r)
            if (r < nrows) (*this)(row0 + r, lane, acc[r]);
    }
    __device__ __forceinline__ void operator()(int row, int lane, double2 acc) const {
        const size_t i = (size_t)row * U + lane;
        const double2 hv = h[(size_t)row * R + lane % R];
        double2 r = c_sub(y[i], acc);
        r = c_add(r, c_mul(hv, u[i]));
        yperf[i] = r;
    }
};

// Perfect-CSI branch of an IC iteration fused into the second pass (select-mode
// schemes whose precoder is row-local, e.g. OFDM): y_perf of the row is formed
// in registers, equalised by the true diag(D), sliced and counted (script:548-561)
// and — unless this is the last iteration — replaced in place by the
// re-precoded decision u = P [xP; Q(x_perf)] (script:541-543).  Pilot rows of u
// are constant (P xP) and are left untouched.  LDS: constellation + slicer.
struct StorePerfectDetect {
    const double2* __restrict__ y;
    const double2* __restrict__ h;     // [LK][R]
    double2* __restrict__ u;           // [LK][U], in/out
    const uint16_t* __restrict__ sidx; // [ND][R]
    const int* __restrict__ row_data;
    const int* __restrict__ row_cons;
    const double2* __restrict__ row_pval;
    const double2* __restrict__ symbols;
    const double* __restrict__ lvI;
    const double* __restrict__ lvQ;
    const int* __restrict__ grid_sym;
    unsigned long long* __restrict__ counters;
    size_t cidx0;                      // counter index of (scheme, csi=1, edge=0, snr=0, stage)
    int cstride_edge, cstride_snr;
    int U, R, snr0, last, M, nI, nQ, real_detect;
    int rvalid;                        // realisations of the batch that count (McBuffers::rvalid)
    double idd, sI, sQ;
    // the chains' folded slicer (nearest_lin): f = z scale + offset, top = n - 1
    double scI, ofI, topI, scQ, ofQ, topQ;
    double rQ;                         // k_pic_fft: scQ / scI (its chain runs on u scI)
    double pf_scale_re, pf_scale_im;   // k_pic_fft: qs gs (SchemeK::pf_scale)
    const double2* xp;                 // pilots [NP][R] (k_mic_pilot: the LS division)
    const double2* xs;                 // precoded symbols P [xP; xD] [LK][R] (the constant rows of v / u)
    const uint16_t* sidr;              // transmitted symbol index per data row [LK][R]
    const TraceK* tr;                  // null unless tracing (dsce_trace_unit_ex)
    int stage;                         // IC iteration of this pass (trace only)
    int pv_uni;                        // chain kernels: SchemeK::pv_uni (reprecode6 / stage_sym)
    double pv_re, pv_im;
    double2* sym;
    SlicerLds* slt;
    int c0, c1;
    __device__ __forceinline__ void prepare(double2* lds) {
        sym = lds;
        slt = (SlicerLds*)(lds + 256);
        constexpr int PER = 256 / WAVE;
        double2 sv[PER];
        int gv[PER];
        const int tid = threadIdx.x;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = tid + k * WAVE;
            sv[k] = i < M ? symbols[i] : make_double2(0.0, 0.0);
            gv[k] = i < nI * nQ ? grid_sym[i] : 0;
        }
        const double li = tid < nI && tid < 16 ? lvI[tid] : 0.0;
        const double lq = tid < nQ && tid < 16 ? lvQ[tid] : 0.0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            sym[tid + k * WAVE] = sv[k];
            slt->grid[tid + k * WAVE] = gv[k];
        }
        if (tid < 16) {
            slt->lvI[tid] = li;
            slt->lvQ[tid] = lq;
        }
        __syncthreads();
        c0 = 0;
        c1 = 0;
    }
    __device__ __forceinline__ void operator()(int row, int lane, double2 acc) {
        if (row_data[row] < 0) return;
        detect(row, lane, acc, u[(size_t)row * U + lane]);
    }
    // Rows in groups of 4: every input of a group (y, h, u, transmitted symbol
    // index, row tables) is requested before the group's first store, so one
    // memory round trip covers four rows instead of one.  ur: the rows' u values
    // if the caller holds them in registers (k_pic), else null.
    template <int RBN>
    __device__ __forceinline__ void rows(int row0, int nrows, int lane, const double2 (&acc)[RBN]) {
        rows_impl<RBN, false>(row0, nrows, lane, acc, acc);
    }
    template <int RBN>
    __device__ __forceinline__ void rows_u(int row0, int nrows, int lane, const double2 (&acc)[RBN],
                                           const double2 (&ur)[RBN]) {
        rows_impl<RBN, true>(row0, nrows, lane, acc, ur);
    }
    template <int RBN, bool UREG>
    __device__ __forceinline__ void rows_impl(int row0, int nrows, int lane, const double2 (&acc)[RBN],
                                              const double2 (&ur)[RBN]) {
        const int rl = lane % R;
#pragma unroll
        for (int g0 = 0; g0 < RBN; g0 += 4) {
            double2 yv[4], hv[4], uv[4], pv[4];
            int tx[4], dd[4], cn[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = g0 + k;
                const int row = row0 + (r < nrows ? r : 0);
                dd[k] = r < nrows ? row_data[row] : -1;
                cn[k] = row_cons[row];
                pv[k] = row_pval[row];
                const size_t i = (size_t)row * U + lane;
                yv[k] = y[i];
                hv[k] = h[(size_t)row * R + rl];
                uv[k] = UREG ? ur[r < RBN ? r : 0] : u[i];
                tx[k] = sidx[(size_t)(dd[k] > 0 ? dd[k] : 0) * R + rl];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = g0 + k;
                if (dd[k] < 0) continue;
                double2 rr = c_sub(yv[k], acc[r < RBN ? r : 0]);
                rr = c_add(rr, c_mul(hv[k], uv[k]));
                const double2 z = c_div1(rr, hv[k]);
                const int dp = slice_fast(*slt, nI, nQ, real_detect ? make_double2(z.x * idd, 0.0)
                                                                    : make_double2(z.x * idd, z.y * idd), sI, sQ);
                const int ne = __popc((unsigned)(dp ^ tx[k]));
                c0 += ne;
                c1 += cn[k] ? ne : 0;
                if (tr && lane == tr->unit) {
                    tr->yperf[(size_t)stage * tr->LK + row0 + r] = rr;
                    tr->dec_p[(size_t)stage * tr->ND + dd[k]] = dp;
                }
                if (!last) {
                    double2 av = make_double2(0.0, 0.0);
                    c_fma(av, pv[k], sym[dp]);
                    u[(size_t)(row0 + r) * U + lane] = av;
                }
            }
        }
    }
    // y_perf = y - acc + h u of one row, sliced, counted, re-precoded into u
    __device__ __forceinline__ void detect(int row, int lane, double2 acc, double2 uv) {
        const size_t i = (size_t)row * U + lane;
        const int rl = lane % R;
        const double2 hv = h[(size_t)row * R + rl];
        const int d = row_data[row];
        if (d < 0) return;
        double2 r = c_sub(y[i], acc);
        r = c_add(r, c_mul(hv, uv));
        const double2 z = c_div1(r, hv);
        const int dp = slice_fast(*slt, nI, nQ, real_detect ? make_double2(z.x * idd, 0.0)
                                                            : make_double2(z.x * idd, z.y * idd), sI, sQ);
        const int ne = __popc((unsigned)(dp ^ (int)sidx[(size_t)d * R + rl]));
        c0 += ne;
        c1 += row_cons[row] ? ne : 0;
        if (tr && lane == tr->unit) {
            tr->yperf[(size_t)stage * tr->LK + row] = r;
            tr->dec_p[(size_t)stage * tr->ND + d] = dp;
        }
        if (!last) {
            double2 av = make_double2(0.0, 0.0);
            c_fma(av, row_pval[row], sym[dp]);
            u[i] = av;
        }
    }
    __device__ __forceinline__ void finish(int lane) {
        const bool valid = lane % R < rvalid;
        const int t0 = wave_sum(valid ? c0 : 0), t1 = wave_sum(valid ? c1 : 0);
        const int l = threadIdx.x & 63;
        if (l < 2) {                                         // one atomic instruction, two lanes
            const int snr = snr0 + (lane - (int)threadIdx.x) / R;
            const size_t i0 = cidx0 + (size_t)snr * cstride_snr + (l ? (size_t)cstride_edge : 0);
            const int v = l ? t1 : t0;
            if (v) atomicAdd(&counters[i0], (unsigned long long)v);
        }
    }
};

// ---------------------------------------------------------------------------
// a7: TX chain, lane = realisation.  Pilots (script:365-368), data symbols from
// bits (script:355-362), x = P [xP; xD] (script:371-373).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_tx_symbols(SchemeK sk, int bits_slot, int pilot_slot, uint64_t seed,
                                                   uint64_t rep0, int R, double2* __restrict__ xp,
                                                   uint16_t* __restrict__ sidx, double2* __restrict__ xs,
                                                   uint16_t* __restrict__ sidr) {
    __shared__ double2 sym[256];
    for (int i = threadIdx.x; i < sk.M; i += WAVE) sym[i] = sk.symbols[i];
    __syncthreads();
    const int rl = blockIdx.x * WAVE + threadIdx.x;
    const uint64_t rep = rep0 + (uint64_t)rl;
    const uint32_t mmask = (uint32_t)(sk.M - 1);
    for (int j = 0; j < sk.NP; ++j) {
        const uint4 w = stream_block(seed, rep, STREAM_PILOTS, pilot_slot, (uint32_t)j >> 2);
        const uint32_t word = (j & 3) == 0 ? w.x : (j & 3) == 1 ? w.y : (j & 3) == 2 ? w.z : w.w;
        const double2 s = sym[word & mmask];
        const double a = hypot(s.x, s.y);
        xp[(size_t)j * R + rl] = make_double2(s.x / a, s.y / a);
    }
    for (int i = 0; i < sk.ND; ++i) {
        const uint32_t q = (uint32_t)(i * sk.mbits);               // first bit of symbol i
        const uint4 w = stream_block(seed, rep, STREAM_BITS, bits_slot, q >> 7);
        const uint32_t wi = (q >> 5) & 3;
        const uint32_t word = wi == 0 ? w.x : wi == 1 ? w.y : wi == 2 ? w.z : w.w;
        const uint16_t si = (uint16_t)((word >> (q & 31)) & mmask);   // bi2de, LSB first
        sidx[(size_t)i * R + rl] = si;
        // the same, row-indexed (select mode only: data_pos holds one dummy entry
        // for a data-spreading scheme, whose data symbols have no rows)
        if (!sk.despread) sidr[(size_t)sk.data_pos[i] * R + rl] = si;
    }
    // x = P [xP; xD]
    for (int r = 0; r < sk.LK; ++r) {
        double2 acc = make_double2(0.0, 0.0);
        for (int j = sk.p_ptr[r]; j < sk.p_ptr[r + 1]; ++j) {
            const int k = sk.p_col[j];
            const double2 xin = k < sk.NP ? xp[(size_t)k * R + rl] : sym[sidx[(size_t)(k - sk.NP) * R + rl]];
            c_fma(acc, sk.p_val[j], xin);
        }
        xs[(size_t)r * R + rl] = acc;
    }
}

// k_tx_symbols for row-local precoders (SchemeK::tx_rows, e.g. OFDM's P): every
// row carries one pilot or data column, so the rows are drawn in parallel,
// S row slices per realisation (grid R/64 x S: 8 waves / SIMD instead of one,
// whose 336 sequential stream draws per lane left it latency-bound at 12 %
// VALU issue).  Same draws, same arithmetic: xp = s / |s|, the data index from
// the bit stream, xs[r] = p_val (0 + xin), sidr[r] = the row's data index.
template <int S>
__global__ void __launch_bounds__(64) k_tx_rows(SchemeK sk, int bits_slot, int pilot_slot, uint64_t seed, uint64_t rep0,
                                                int R, double2* __restrict__ xp, uint16_t* __restrict__ sidx,
                                                double2* __restrict__ xs, uint16_t* __restrict__ sidr) {
    __shared__ double2 sym[256];
    for (int i = threadIdx.x; i < sk.M; i += WAVE) sym[i] = sk.symbols[i];
    __syncthreads();
    const int rl = blockIdx.x * WAVE + threadIdx.x;
    const uint64_t rep = rep0 + (uint64_t)rl;
    const uint32_t mmask = (uint32_t)(sk.M - 1);
    for (int r = blockIdx.y; r < sk.LK; r += S) {
        const int k = sk.row_pcol[r];                          // uniform: one row per block and step
        double2 acc = make_double2(0.0, 0.0);
        if (k >= 0 && k < sk.NP) {
            const uint4 w = stream_block(seed, rep, STREAM_PILOTS, pilot_slot, (uint32_t)k >> 2);
            const uint32_t word = (k & 3) == 0 ? w.x : (k & 3) == 1 ? w.y : (k & 3) == 2 ? w.z : w.w;
            const double2 s = sym[word & mmask];
            const double a = hypot(s.x, s.y);
            const double2 pv = make_double2(s.x / a, s.y / a);
            xp[(size_t)k * R + rl] = pv;
            c_fma(acc, sk.row_pval[r], pv);
        } else if (k >= sk.NP) {
            const int i = k - sk.NP;
            const uint32_t q = (uint32_t)(i * sk.mbits);
            const uint4 w = stream_block(seed, rep, STREAM_BITS, bits_slot, q >> 7);
            const uint32_t wi = (q >> 5) & 3;
            const uint32_t word = wi == 0 ? w.x : wi == 1 ? w.y : wi == 2 ? w.z : w.w;
            const uint16_t si = (uint16_t)((word >> (q & 31)) & mmask);
            sidx[(size_t)i * R + rl] = si;
            sidr[(size_t)r * R + rl] = si;
            c_fma(acc, sk.row_pval[r], sym[si]);
        }
        xs[(size_t)r * R + rl] = acc;
    }
}

// r0 = H s (script:383-385), lane = realisation, grid (R/64, ceil(N/64)).
__global__ void __launch_bounds__(64) k_channel_apply(ChannelK ch, int R, const double2* __restrict__ ir,
                                                      const double2* __restrict__ ss, double2* __restrict__ r0) {
    const int rl = blockIdx.x * WAVE + threadIdx.x;
    const int n0 = blockIdx.y * 64;
    for (int n = n0; n < n0 + 64 && n < ch.N; ++n) {
        double2 acc = make_double2(0.0, 0.0);
        for (int q = 0; q < ch.ntap; ++q) {
            const int m = n - ch.tap_delay[q];
            if (m >= 0) c_fma(acc, ir[((size_t)q * ch.N + n) * R + rl], ss[(size_t)m * R + rl]);
        }
        r0[(size_t)n * R + rl] = acc;
    }
}

void launch_tx(hipStream_t s, const SchemeK& sk, const ChannelK& ch, int bits_slot, int pilot_slot, uint64_t seed,
               uint64_t rep0, McBuffers& b, bool txrx, bool rows) {
    const int R = b.R;
    if (sk.tx_rows && rows)
        hipLaunchKernelGGL((k_tx_rows<8>), dim3(R / WAVE, 8), dim3(WAVE), 0, s, sk, bits_slot, pilot_slot, seed, rep0,
                           R, b.xp, b.sidx, b.xs, b.sidr);
    else
        hipLaunchKernelGGL(k_tx_symbols, dim3(R / WAVE), dim3(WAVE), 0, s, sk, bits_slot, pilot_slot, seed, rep0, R,
                           b.xp, b.sidx, b.xs, b.sidr);
    if (txrx) return;      // s, r0 and diag(D) come from k_txrx_fft with the receiver front
    // s = G x (script:376-378)
    launch_band(s, sk.G, R, nullptr, LoadSoA{b.xs, R}, StoreSoA{b.ss, R});
    hipLaunchKernelGGL(k_channel_apply, dim3(R / WAVE, (ch.N + 63) / 64), dim3(WAVE), 0, s, ch, R, b.ir, b.ss, b.r0);
    // a8: h = diag(Q' H G) (script:388-393) without forming D: banded matvec over the taps
    launch_band(s, sk.HD, R, nullptr, LoadTapInterleaved{b.ir, ch.N, R, ch.ntap}, StoreSoA{b.h, R});
}

// ---------------------------------------------------------------------------
// a12: r = r0 + noise (script:397-403), lane = unit; grid (U/64, ceil(N/64)).
// Noise sub-stream k + 256 * slot with k = base + snr the SNR point's index in
// the full sweep (Opts::snr_base: a rank serving SNR points [base, ...) of a
// sweep draws the one-rank run's noise) and slot the noise slot (schemes drawing
// separate noise, e.g. n_FBMC / n_OFDM of SimpleVersion_DoublyFlat.m:125-126).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_noise(int N, int R, int U, int snr0, int slot, int base, const double* __restrict__ pn, uint64_t seed,
                                              uint64_t rep0, const double2* __restrict__ r0,
                                              double2* __restrict__ rbuf) {
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int snr = snr0 + unit / R, rl = unit % R;
    const uint64_t rep = rep0 + (uint64_t)rl;
    const double sc = sqrt(pn[snr] / 2.0);
    const int n0 = blockIdx.y * 64;
    for (int n = n0; n < n0 + 64 && n < N; ++n) {
        const uint4 w = stream_block(seed, rep, STREAM_NOISE, (uint32_t)(base + snr + 256 * slot), (uint32_t)n);
        rbuf[(size_t)n * U + unit] = noise_add(r0[(size_t)n * R + rl], sc, w);
    }
}

// r = r0 + noise generated on the fly as the column operand of the Q^H band
// (the noise of k_noise, bit for bit, but only for the samples Q^H reads — the
// OFDM cyclic prefixes and zero guards are never drawn — and r never touches
// memory).  Used when every sample feeds at most one Q^H row block.
struct LoadNoisy {
    const double2* __restrict__ r0;    // [N][R]
    const double* __restrict__ pn;
    uint64_t seed, rep0;
    int R, snr0, slot, base;
    typedef double2 Regs;
    __device__ __forceinline__ Regs load(int n, int lane) const {
        const int snr = snr0 + lane / R, rl = lane % R;
        const double sc = sqrt(pn[snr] / 2.0);
        const uint4 w = stream_block(seed, rep0 + (uint64_t)rl, STREAM_NOISE, (uint32_t)(base + snr + 256 * slot),
                                     (uint32_t)n);
        return noise_add(r0[(size_t)n * R + rl], sc, w);
    }
    __device__ __forceinline__ double2 combine(const Regs& r) const { return r; }
};

static unsigned launch_txrx(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, const double* pn,
                            uint64_t seed, uint64_t rep0, McBuffers& b);

unsigned launch_rx_front(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, const double* pn,
                         uint64_t seed, uint64_t rep0, McBuffers& b) {
    if (txrx_fft_ok(op, sk, ch, b)) return launch_txrx(s, op, sk, ch, pn, seed, rep0, b);
    if (sk.qh_disjoint && op.noise_fuse) {
        launch_band(s, sk.QH, b.U, nullptr, LoadNoisy{b.r0, pn, seed, rep0, b.R, b.snr0, sk.noise_slot, op.snr_base},
                    StoreSoA{b.y, b.U});
        return PATH_NOISE_FUSED;
    }
    hipLaunchKernelGGL(k_noise, dim3(b.U / WAVE, (sk.N + 63) / 64), dim3(WAVE), 0, s, sk.N, b.R, b.U, b.snr0, sk.noise_slot,
                       op.snr_base, pn, seed, rep0,
                       b.r0, b.t);
    // y = Q' r (script:406-409)
    launch_band(s, sk.QH, b.U, nullptr, LoadSoA{b.t, b.U}, StoreSoA{b.y, b.U});
    return 0;
}

typedef double d4 __attribute__((ext_vector_type(4)));

#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)


// Raw buffer view of a wave-uniform base (T8): a 32-bit per-lane byte offset plus
// a wave-uniform one (SGPR) per load instead of 64-bit address arithmetic.
// Callers keep every access inside the allocation (no reliance on the range check).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                             (int)(unsigned)(bytes < 0xFFFFFFFFull ? bytes : 0xFFFFFFFFull), 0x00020000);
}
__device__ __forceinline__ double2 buf_ld2(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    return make_double2(__hiloint2double((int)v.y, (int)v.x), __hiloint2double((int)v.w, (int)v.z));
}
__device__ __forceinline__ unsigned buf_ldu16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
}
// The per-unit rows 4 a + r (a = 0..5) of one 24-row symbol block of a [LK][ld]
// array: a buffer view from the block's first row, the lane's byte offset
// (r ld + col) esz, and row a at the wave-uniform offset 4 a ld esz (SGPR): no
// 64-bit address arithmetic per load (r05; the chain kernels' prologues spent
// ~3 VALU per row and array on it).  Callers: 24 ld esz < 2^32 (pic_fft_ok).
struct RowView {
    __amdgpu_buffer_rsrc_t rs;
    unsigned voff, step;
    __device__ __forceinline__ RowView(const void* base, int row0, int ld, int r, int col, int esz) {
        rs = buf_rsrc((const char*)base + (size_t)row0 * ld * esz, (size_t)24 * ld * esz);
        voff = (unsigned)(r * ld + col) * (unsigned)esz;
        step = 4u * (unsigned)ld * (unsigned)esz;
    }
    __device__ __forceinline__ double2 ld2(int a) const { return buf_ld2(rs, voff, (unsigned)a * step); }
    __device__ __forceinline__ unsigned ldu16(int a) const { return buf_ldu16(rs, voff, (unsigned)a * step); }
};

// Nearest level of a uniform level grid lv0 + i step (i < n) by rounding
// f = (x - lv0) / step + 0.5, folded into one FMA.  An exact mid-point (f
// integral, inside the grid) flags the lower neighbour as the tie alternative
// (first-minimum rule of SignalConstellation.m:88, resolved on the grid by the
// caller: a flag at level 0 reads level 0 twice); NaN / inf (h == 0) clamp into
// the grid.  The clamp runs on the truncated integer (v_cvt_i32_f64 saturates
// and maps NaN to 0; below 0 truncation and floor clamp alike): two f64 ops
// per component fewer than floor / fmax / fmin.
__device__ __forceinline__ int nearest_lin(double x, double scale, double offset, double top, int& tie) {
    const double f = fma(x, scale, offset);              // (x - lv0) / step + 0.5
    int t, c;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(t) : "v"(f));
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(c) : "v"(t), "v"((int)top));
    tie = f == (double)c ? 1 : 0;                        // on the mid-point below level c
    return c;
}

// The folded slicer of the chain kernels for the lane's six rows (r05): f = z
// scale + offset per component (nearest_lin's), nearest grid indices by
// truncation + clamp, symbol from the LDS grid.  An exact mid-point needs f to
// be an integer below 2^20, so the low word of f is zero: that one integer
// compare per component flags the (measure-zero) candidates, and the exact test
// f == (double)c with the first-minimum rule of SignalConstellation.m:88 runs
// only in the rare branch it takes (r04: a conversion back and an FP64 compare
// per component and row, 24 FP64 instructions per six rows).
__device__ __forceinline__ int nearest_idx(double f, double top) {
    int t, c;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(t) : "v"(f));
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(c) : "v"(t), "v"((int)top));
    return c;
}
// g8: the level-grid -> symbol map as bytes at [iI][iQ] with row stride 16
// (nI, nQ <= 16, M <= 256): the LDS address is one shift-or (r05; an int
// table at iI nQ + iQ took a multiply and two shifts per row)
__device__ __forceinline__ void slice6(int (&dp)[6], const double (&fI)[6], const double (&fQ)[6], double topI,
                                       double topQ, const unsigned char* g8) {
    int code[6];
    // candidates: any low word zero, by one unsigned min over the twelve words
    // (v_min3_u32 chain; r05 — per-word compares cost ~35 instructions)
    unsigned lo = 0xffffffffu;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const int iI = nearest_idx(fI[a], topI), iQ = nearest_idx(fQ[a], topQ);
        code[a] = iI | (iQ << 8);
        lo = min(lo, min((unsigned)__double2loint(fI[a]), (unsigned)__double2loint(fQ[a])));
        dp[a] = g8[(iI << 4) | iQ];
    }
    if (__ballot(lo == 0u)) {
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            // opaque copies: the exact test stays inside the rare branch (if-
            // converted, the compiler evaluated it for every row)
            double gI = fI[a], gQ = fQ[a];
            asm volatile("" : "+v"(gI), "+v"(gQ));
            const int iI = code[a] & 0xff, iQ = (code[a] >> 8) & 0xff;
            const int jI = max(iI - (gI == (double)iI ? 1 : 0), 0), jQ = max(iQ - (gQ == (double)iQ ? 1 : 0), 0);
            dp[a] = min(min((int)g8[(iI << 4) | iQ], (int)g8[(jI << 4) | iQ]),
                        min((int)g8[(iI << 4) | jQ], (int)g8[(jI << 4) | jQ]));
        }
    }
}

// u of the lane's data rows <- the re-precoded decisions P [.; x_hat] (row-local
// P): the row's precoder value times the decided symbol.  pv_uni (SchemeK): every
// data row has the same value and the staged constellation (stage_sym) already
// carries it, so the product is one LDS read (a uniform branch).
__device__ __forceinline__ void reprecode6(double2 (&u)[6], const int (&dp)[6], unsigned dmask, const double2* rpv, int r,
                                           const double2* sym, int pv_uni) {
    if (pv_uni) {
        // every row reads its entry (dp is a valid index on every row): without the
        // opaque copy the compiler turned each select into a per-row branch around
        // the LDS read, each with its own wait (DESIGN.md lesson 4)
        double2 nv[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) nv[a] = sym[dp[a]];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            asm volatile("" : "+v"(nv[a].x), "+v"(nv[a].y));
            const bool data = (dmask >> a) & 1;
            u[a].x = data ? nv[a].x : u[a].x;
            u[a].y = data ? nv[a].y : u[a].y;
        }
    } else {
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const bool data = (dmask >> a) & 1;
            double2 nv = make_double2(0.0, 0.0);
            c_fma(nv, rpv[4 * a + r], sym[dp[a]]);
            u[a].x = data ? nv.x : u[a].x;
            u[a].y = data ? nv.y : u[a].y;
        }
    }
}
// constellation entry i as staged for reprecode6: times the common data-row
// precoder value when pv_uni (the very product reprecode6 forms otherwise)
__device__ __forceinline__ double2 stage_sym(double2 a, int pv_uni, double pvr, double pvi) {
    if (!pv_uni) return a;
    double2 nv = make_double2(0.0, 0.0);
    c_fma(nv, make_double2(pvr, pvi), a);
    return nv;
}

// Error counts of a 256-thread block, one atomic per counter per block: every
// wave packs its totals (errors | no-edge errors << 16, per CSI branch) and
// wave 0 sums the four waves' words from LDS.  `words` = 1 or 2 branches.
// valid: as flush_mse.
__device__ __forceinline__ void block_counts(const int (&packed)[2], int words, int* lds /* [4][2] */,
                                             unsigned long long* counters, size_t base, size_t stride_edge,
                                             size_t stride_csi, bool valid) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int t0 = wave_sum(valid ? packed[0] : 0);
    const int t1 = words > 1 ? wave_sum(valid ? packed[1] : 0) : 0;
    if (l == 0) {
        lds[2 * w] = t0;
        lds[2 * w + 1] = t1;
    }
    __syncthreads();
    if (threadIdx.x < 2 * words) {
        const int csi = threadIdx.x >> 1, edge = threadIdx.x & 1;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v += (lds[2 * k + csi] >> (16 * edge)) & 0xffff;
        if (v) atomicAdd(&counters[base + csi * stride_csi + edge * stride_edge], (unsigned long long)v);
    }
}

// IC iterations per chain launch (k_pic_fft, k_mic_fft): the per-iteration
// error counts of a wave go through LDS and are added once at the end.
static constexpr int PM_MAXIT = 32;

// ---------------------------------------------------------------------------
// The perfect-CSI IC chain of OFDM by FFT on the VALU (k_pic_fft, SchemeK::pf_ok).
// For OFDM with FFT size = subcarriers = 24 and no intermediate frequency, the
// Q^H block of symbol k is qs * DFT and its G block is gs * IDFT with a cyclic
// prefix (OFDM.m GetTXMatrix / GetRXMatrix; pack_scheme verifies every entry),
// so (Q'HG u)_blk = qs gs FFT24(h_0 .* t + h_1 .* t(-1)), t = IFFT24(u): ~10x
// fewer flops than two dense 24 x 24 products on the matrix cores (the r01
// k_pic_mfma) — and on gfx950 f64 MFMA and VALU work do not overlap
// (profiles/r02_mfma_valu_overlap.txt), so the flop count is what matters.
// ---------------------------------------------------------------------------
__constant__ double2 kW24[12] = {
    {1.0, 0.0},
    {0.96592582628906829, 0.25881904510252076},
    {0.86602540378443865, 0.5},
    {0.70710678118654752, 0.70710678118654752},
    {0.5, 0.86602540378443865},
    {0.25881904510252076, 0.96592582628906829},
    {0.0, 1.0},
    {-0.25881904510252076, 0.96592582628906829},
    {-0.5, 0.86602540378443865},
    {-0.70710678118654752, 0.70710678118654752},
    {-0.86602540378443865, 0.5},
    {-0.96592582628906829, 0.25881904510252076}};

// x * (c + S i s) for compile-time c, s
template <int S>
__device__ __forceinline__ double2 cmul_const(double2 x, double c, double s) {
    return make_double2(fma(x.x, c, -(S * s) * x.y), fma(x.y, c, (S * s) * x.x));
}

// DFT-3 with sign S (S = +1: sum x[n] e^{+2 pi i nk/3}); the +-i H (b - c)
// rotation fused into the output FMAs (12 FP64 ops)
template <int S>
__device__ __forceinline__ void dft3(double2& a, double2& b, double2& c) {
    constexpr double H = 0.86602540378443865;           // sin(60 deg)
    const double2 t = c_add(b, c), d = c_sub(b, c);
    const double2 m = make_double2(fma(-0.5, t.x, a.x), fma(-0.5, t.y, a.y));
    a = c_add(a, t);
    b = make_double2(fma(-S * H, d.y, m.x), fma(S * H, d.x, m.y));   // m + S i H d
    c = make_double2(fma(S * H, d.y, m.x), fma(-S * H, d.x, m.y));   // m - S i H d
}

// a * b with two FMAs (2 mul + 2 fma instead of 4 mul + 2 add under -ffp-contract=off)
__device__ __forceinline__ double2 c_mulf(double2 a, double2 b) {
    return make_double2(fma(a.x, b.x, -(a.y * b.y)), fma(a.x, b.y, a.y * b.x));
}

// e * w of the quad network's middle twiddle: 1 on lanes 0-2, +i (S = 1, forward)
// or -i (S = -1, inverse) on lane 3 -- as selects (five 32-bit ops) instead of a
// complex product (four f64 ops)
template <int S>
__device__ __forceinline__ double2 quad_tw(double2 e, bool r3) {
    const double nx = S > 0 ? -e.y : e.y, ny = S > 0 ? e.x : -e.x;
    return make_double2(r3 ? nx : e.x, r3 ? ny : e.y);
}


// D = A B of the four 4 x 4 blocks of v_mfma_f64_4x4x4f64 with complex A and B
// (this lane's entries a, b): re = Ar Br - Ai Bi, im = Ar Bi + Ai Br, two
// accumulating MFMAs each
__device__ __forceinline__ double2 mfma4_cmul(double2 a, double2 b) {
    double re = __builtin_amdgcn_mfma_f64_4x4x4f64(a.x, b.x, 0.0, 0, 0, 0);
    // - Ai Bi by the f64 MFMA's neg modifier on A (the blgp field on gfx950,
    // neg:[1,0,0]) instead of two VALU moves per product (r05)
    re = __builtin_amdgcn_mfma_f64_4x4x4f64(a.y, b.y, re, 0, 0, 1);
    double im = __builtin_amdgcn_mfma_f64_4x4x4f64(a.x, b.y, 0.0, 0, 0, 0);
    im = __builtin_amdgcn_mfma_f64_4x4x4f64(a.y, b.x, im, 0, 0, 0);
    return make_double2(re, im);
}

// a complex from lane addr / 4 of the wave (ds_bpermute: the LDS crossbar, no LDS
// allocation, no barrier)
__device__ __forceinline__ double2 bperm_c(int addr, double2 v) {
    return make_double2(__hiloint2double(__builtin_amdgcn_ds_bpermute(addr, __double2hiint(v.x)),
                                         __builtin_amdgcn_ds_bpermute(addr, __double2loint(v.x))),
                        __hiloint2double(__builtin_amdgcn_ds_bpermute(addr, __double2hiint(v.y)),
                                         __builtin_amdgcn_ds_bpermute(addr, __double2loint(v.y))));
}

// position of output k of dft6 in the array: X[k] lands at x[-k mod 6]
__host__ __device__ constexpr int p6(int k) { return (6 - k) % 6; }

// DFT-6 with sign S in place, natural-order input, output k at x[p6(k)]
// (r05): Good-Thomas prime-factor form, 6 = 2 x 3 coprime, so no twiddles:
// n = 3 n1 + 2 n2, k = 3 k1 + 4 k2 (mod 6); DFT-3 over n2 of (x0, x2, x4) and
// (x3, x5, x1), then DFT-2 over n1: 36 FP64 ops instead of 48 (r04: DFT-3 x 2,
// twiddles w6^1 / w6^2, DFT-2 x 3)
template <int S>
__device__ __forceinline__ void dft6(double2 (&x)[6]) {
    dft3<S>(x[0], x[2], x[4]);
    dft3<S>(x[3], x[5], x[1]);
    // pairs (A0[k2], A1[k2]) = (x0, x3), (x2, x5), (x4, x1) -> X[4 k2], X[4 k2 + 3]
#pragma unroll
    for (int k2 = 0; k2 < 3; ++k2) {
        const int i0 = 2 * k2, i1 = (2 * k2 + 3) % 6;
        const double2 a = x[i0], b = x[i1];
        x[i0] = c_add(a, b);
        x[i1] = c_sub(a, b);
    }
}

// k_pic_fft: a lane QUAD owns a unit.  Lane r holds the rows 4a + r (a = 0..5)
// — u (the decisions), the iteration-invariant y / h and 1 / h, and the channel
// taps of its samples, all in registers, so the iteration loop reads no memory
// — and, in the time domain, the samples 6c + m' with c = bitrev2(r).  DFT-24 =
// DFT-6 per lane x a radix-2 x 2 network across the quad (DPP quad_perm), lane
// twiddles w24^(r m') from LDS; the output scale qs gs is folded into the
// forward twiddles.  One-tap z = y_perf / h = y / h - acc / h + u.
// 198 VGPRs, 2 waves / SIMD (3 waves forced spills or per-iteration reloads of
// y, h and the taps: 4.45 / 5.25 ms vs 2.57 ms per 65536-realisation launch).
// Block = 256 threads = 64 units of one symbol; grid: symbols x units/64,
// SNR-fastest XCD-aware order.
// S0 (r03, with k_mic_pilot / k_mic_data): the chain also runs stage 0 of the
// perfect-CSI branch, the one-tap x = y ./ h (script:450-466), so no stage
// kernel runs in front: u starts as P [xP; 0] (xs of the pilot rows) and the
// data rows get the stage-0 decisions in registers.
// NM (r03k): the 4-point network on the matrix cores instead.  A unit's four
// quarters sit on the four 16-lane rows (lane = 16 r + unit), which is the K
// index of v_mfma_f64_4x4x4f64 (4 blocks of 4 units: B[k][n] in lane 16 k +
// 4 c + n, D[i][n] in lane 16 i + 4 c + n, A[i][k] in lane 16 k + 4 c + i), so
// per sample m the whole network including the lane twiddle is one complex
// 4 x 4 product, A_m[i][k] = i^(i k) w24^(k m) (inverse) or qs gs i^(-i k)
// w24^(-i m) (forward; outputs in natural order): four MFMAs (re / im x the
// two real K halves, 72 cycles per m per wave on the box) instead of the lane
// twiddle, 8 DPP moves, 4 FMAs and the +-i selects (100 cycles,
// tools/ubench/net.hip).  The previous quarter's sample 5 comes by ds_bpermute.
// r05 (the per-section census, profiles/r05_census_*): the iteration carried
// ~40 register copies (the loop state of the fixed-point exit, option pic_skip,
// retired in r06), the imaginary A parts were negated by VALU moves (now the f64 MFMA's
// neg modifier, mfma4_cmul), the tie candidates took ~35 instructions per
// iteration (now one min3 chain), and the epilogue spent 10 FP64 operations
// per row.  The chain now runs on u scaled by the slicer's scale c = scI: the
// transforms are linear, so acc = c D u, and with Yo = c y / h + (ofI, 0) the
// folded slicer input is
//   fI = Yo.x + us.x - (acc / h).x,  fQ = (Yo.y + us.y - (acc / h).y) scQ / scI + ofQ
// (7 FP64 operations per row; r06: the taps are centred over the window, acc =
// c (D - diag h) u, and the us terms go: 5).  Re-precoded decisions read the scaled
// constellation; the constant rows of u (pilots) are per-lane LDS slots read
// through the same address select, so a row's new u is one LDS read.
// (vb / vn = the block's index in the grid and the grid's size, vb % 8 = the XCD)
template <int NT, int SH, bool TRACE, bool S0, bool NM>
__device__ __forceinline__ void pic_fft_body(const SchemeK& sk, const BandOrder& ord, const double2* __restrict__ ir, int N,
                                             const StorePerfectDetect& o, int niter, int vb, int vn) {
    int ug, blk;
    band_block(ord, sk.QH.nblk, ug, blk, vb, vn);
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = NM ? l >> 4 : l & 3;
    const int U = o.U, R = o.R;
    const int unit = ug * WAVE + w * 16 + (NM ? (l & 15) : (l >> 2));
    const int rl = unit % R;
    const int cq = NM ? r : (r >> 1) + 2 * (r & 1);            // time quarter of this lane
    const int row0 = sk.QH.row0[blk], klo = sk.QH.klo[blk];
    const double cs = o.scI, rq = o.rQ;                        // the chain's scale (host: scI != 0), scQ / scI
    __shared__ double2 sym[256];
    __shared__ unsigned sgridw[64];                            // slice6's byte grid as words
    const unsigned char* sgrid = (const unsigned char*)sgridw;
    __shared__ double2 rpv[24];
    __shared__ int rdc[24];
    __shared__ double2 twa[2][4][6];                            // [IFFT / FFT][lane r][m']
    __shared__ double2 amt[NM ? 2 : 1][6][16];                  // NM: A_m[i][k] at [dir][m][i + 4 k]
    __shared__ int cntl[4][PM_MAXIT + 1];                      // [wave][stage]
    __shared__ double2 ucst[6][256];                            // the lane's constant rows of u (scaled)
    // decisions u (scaled) and the iteration-invariant Yo and 1 / h of the lane's
    // rows, and the channel taps of the lane's samples (registers for all iterations)
    double2 u[6], yh[6], hc[6];
    unsigned txp[2] = {0u, 0u};
    double2 taps[6][NT];
    const __amdgpu_buffer_rsrc_t trs =
        buf_rsrc(ir + (size_t)klo * R, ((size_t)(NT - 1) * N + (N - klo)) * R * sizeof(double2));
    const unsigned tv0 = (unsigned)(6 * cq * R + rl) * 16u;
    {
        // table loads, then the per-unit loads (raw y and h into yh / hc), then
        // the LDS writes: the writes wait only for the tables (vmcnt retires in
        // order), the per-unit data arrives during the barrier.  r06: the tables
        // come precomputed per scheme (SchemeK::ct_*, build_chain_tables), thread
        // t copies entry t (clamped, unconditional: threads past a table's end
        // rewrite its last entry with the same value)
        const double2 a = sk.ct_symc[tid];
        const unsigned gw = sk.ct_grid[min(tid, 63)];
        const int rt = min(tid, 23);
        const double2 pv = sk.ct_rpv[blk * 24 + rt];
        const int rdv = sk.ct_rdc[blk * 24 + rt];
        const double2 nt = NM ? sk.ct_amt[min(tid, 191)] : sk.ct_twa[min(tid, 47)];
        const RowView vu = S0 ? RowView(o.xs, row0, R, r, rl, 16) : RowView(o.u, row0, U, r, unit, 16);
        const RowView vs(o.sidr, row0, R, r, rl, 2), vy(o.y, row0, U, r, unit, 16), vh(o.h, row0, R, r, rl, 16);
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            u[b] = vu.ld2(b);
            txp[b >> 2] |= (vs.ldu16(b) & 0xffu) << (8 * (b & 3));
            yh[b] = vy.ld2(b);
            hc[b] = vh.ld2(b);
        }
#pragma unroll
        for (int m = 0; m < 6; ++m)
#pragma unroll
            for (int q = 0; q < NT; ++q) taps[m][q] = buf_ld2(trs, tv0, (unsigned)((q * N + m) * R) * 16u);
        sym[tid] = a;
        sgridw[min(tid, 63)] = gw;
        rpv[rt] = pv;
        rdc[rt] = rdv;
        if (!NM) (&twa[0][0][0])[min(tid, 47)] = nt;
        else (&amt[0][0][0])[min(tid, 191)] = nt;
    }
    __syncthreads();
    // the taps minus their window mean (r06): a tap constant over the FFT window
    // maps to the diagonal of Q' H G, so the chain now forms (D - diag h) u
    // itself and the one-tap input is y / h - acc / h (no + u per row and
    // iteration); the mean over the unit's four quarters by the all-ones MFMA
    // (NM: quarters on the K rows) or two DPP exchanges (quad layout)
#pragma unroll
    for (int q = 0; q < NT; ++q) {
        double2 sq = taps[0][q];
#pragma unroll
        for (int m = 1; m < 6; ++m) sq = c_add(sq, taps[m][q]);
        if (NM) {
            sq = make_double2(__builtin_amdgcn_mfma_f64_4x4x4f64(1.0, sq.x, 0.0, 0, 0, 0),
                              __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, sq.y, 0.0, 0, 0, 0));
        } else {
            sq = c_add(sq, dpp_c<QP_XOR1>(sq));
            sq = c_add(sq, dpp_c<QP_XOR2>(sq));
        }
        const double2 mq = make_double2(sq.x * (1.0 / 24.0), sq.y * (1.0 / 24.0));
#pragma unroll
        for (int m = 0; m < 6; ++m) taps[m][q] = c_sub(taps[m][q], mq);
    }
    // u scaled by c; the constant rows into the lane's own LDS slots (every row:
    // the data rows' slots are never read; no barrier, only this lane reads them)
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        u[a] = make_double2(u[a].x * cs, u[a].y * cs);
        ucst[a][tid] = u[a];
    }
    // data / no-edge masks of the lane's rows
    unsigned dmask = 0u, emask = 0u;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const int dc = rdc[4 * a + r];
        dmask |= dc >= 0 ? 1u << a : 0u;
        emask |= dc >= 0 && (dc & 1) ? 1u << a : 0u;
    }
    const double sg1 = (r >> 1) ? -1.0 : 1.0, sg2 = (r & 1) ? -1.0 : 1.0;
    int ncnt = 0;
    // error-count weight of row a: data rows count 1, no-edge rows also 1 << 16
    auto cweight = [&](int a) -> int {
        return ((dmask >> a) & 1) ? (((emask >> a) & 1) ? 0x10001 : 1) : 0;
    };
    // the re-precoded decisions (pv_uni): one LDS read per row, the data rows
    // from the scaled constellation, the others from their constant slot
    // (neither branch reads the old u: with reprecode6's selects in the other
    // branch the merge cost 13 register copies per iteration)
    auto reprecode = [&](const int (&dp)[6]) {
        double2 nv[6];
        if (o.pv_uni) {
#pragma unroll
            for (int a = 0; a < 6; ++a) nv[a] = ((dmask >> a) & 1) ? sym[dp[a]] : ucst[a][tid];
        } else {
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double2 pr = c_mulf(rpv[4 * a + r], sym[dp[a]]), cv = ucst[a][tid];
                nv[a] = ((dmask >> a) & 1) ? pr : cv;
            }
        }
#pragma unroll
        for (int a = 0; a < 6; ++a) u[a] = nv[a];
    };
    if (S0) {
        // stage 0: Yo = c y / h + (ofI, 0) and 1 / h now, one-tap, slicer,
        // counts, decisions
        int dp[6];
        double fI[6], fQ[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double2 hh = hc[a], yv = yh[a];
            const double id = recip_fast(hh.x * hh.x + hh.y * hh.y);
            hc[a] = make_double2(hh.x * id, -hh.y * id);
            const double2 ys = c_mulf(yv, hc[a]);
            yh[a] = make_double2(fma(ys.x, cs, o.ofI), ys.y * cs);
            fI[a] = yh[a].x;
            fQ[a] = fma(yh[a].y, rq, o.ofQ);
        }
        slice6(dp, fI, fQ, o.topI, o.topQ, sgrid);
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const bool data = (dmask >> a) & 1;
            ncnt += __umul24(__popc((unsigned)(dp[a] ^ (int)((txp[a >> 2] >> (8 * (a & 3))) & 0xffu))), cweight(a));
            if (TRACE && data && unit == o.tr->unit) o.tr->dec_p[(size_t)(rdc[4 * a + r] >> 1)] = dp[a];
        }
        reprecode(dp);
        cntl[w][0] = wave_sum_dpp(rl < o.rvalid ? ncnt : 0);
        ncnt = 0;
    }
    for (int it = 1; it <= niter; ++it) {
        // an opaque zero keeps the per-iteration LDS twiddle reads inside the loop
        // (hoisted, they would hold 56 more registers)
        int oz = 0;
        asm volatile("" : "+v"(oz));
        const int ro = r + oz;
        // t = IDFT24(u): DFT-6 per lane, twiddle w24^(r m'), 4-point network
        // across the quad (xor 2, lane twiddle, xor 1): lane r ends with the time
        // samples 6 cq + m'
        double2 x[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) x[a] = u[a];
        dft6<1>(x);
        double2 t[6];
        const int ai = (l & 3) + 4 * (l >> 4) + oz;             // NM: this lane's A entry
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            if (NM) {
                const double2 am = amt[0][m][ai], b = x[p6(m)];
                t[m] = mfma4_cmul(am, b);
            } else {
                const double2 p = c_mulf(x[p6(m)], twa[0][ro][m]);
                const double2 pv = dpp_c<QP_XOR2>(p);
                double2 e = make_double2(fma(sg1, p.x, pv.x), fma(sg1, p.y, pv.y));
                e = quad_tw<1>(e, r == 3);
                const double2 qv = dpp_c<QP_XOR1>(e);
                t[m] = make_double2(fma(sg2, e.x, qv.x), fma(sg2, e.y, qv.y));
            }
        }
        // channel, in place, last sample first: x[m] = sum_q IR_q[m] t[m - d_q];
        // t[-1] of the quarter is sample 5 of the previous quarter's lane (the
        // cyclic prefix for quarter 0)
        const double2 tprev = NM ? bperm_c(((l + 48) & 63) * 4, t[5]) : dpp_c<QP_PREV>(t[5]);
#pragma unroll
        for (int m = 5; m >= 0; --m) {
            const double2 tp = m ? t[m - 1] : tprev;
            double2 acc = make_double2(0.0, 0.0);
#pragma unroll
            for (int q = 0; q < NT; ++q) c_fma(acc, taps[m][q], ((SH >> q) & 1) ? tp : t[m]);
            t[m] = acc;
        }
        // acc = qs gs DFT24(x): network across the quad (xor 1, lane twiddle,
        // xor 2) back to lane r = output residue, twiddle qs gs w24^-(r m'), DFT-6
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            if (NM) {
                x[m] = mfma4_cmul(amt[NM ? 1 : 0][m][ai], t[m]);
            } else {
                const double2 pv = dpp_c<QP_XOR1>(t[m]);
                double2 f = make_double2(fma(sg2, t[m].x, pv.x), fma(sg2, t[m].y, pv.y));
                f = quad_tw<-1>(f, r == 3);
                const double2 qv = dpp_c<QP_XOR2>(f);
                x[m] = c_mulf(make_double2(fma(sg1, f.x, qv.x), fma(sg1, f.y, qv.y)), twa[1][ro][m]);
            }
        }
        dft6<-1>(x);
        // Yo and hcs at the first epilogue (not before the loop): the first chain
        // runs while y and h are still in flight (S0: formed above)
        if (it == 1 && !S0)
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double2 hh = hc[a], yv = yh[a];
                const double id = recip_fast(hh.x * hh.x + hh.y * hh.y);
                hc[a] = make_double2(hh.x * id, -hh.y * id);        // 1 / h
                const double2 ys = c_mulf(yv, hc[a]);
                yh[a] = make_double2(fma(ys.x, cs, o.ofI), ys.y * cs); // c y / h + (ofI, 0)
            }
        // epilogue per row 4a + r: the folded slicer input of z = y / h - acc / h
        // (acc = c (D - diag h) u: centred taps), slicer, counts, re-precoded
        // decision into u
        int dp[6];
        double fI[6], fQ[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double2 xa = x[p6(a)], hh = hc[a];
            fI[a] = fma(-xa.x, hh.x, fma(xa.y, hh.y, yh[a].x));
            fQ[a] = fma(fma(-xa.x, hh.y, fma(-xa.y, hh.x, yh[a].y)), rq, o.ofQ);
            if (TRACE && ((dmask >> a) & 1) && unit == o.tr->unit) {
                const int row = row0 + 4 * a + r;
                const double2 yv = o.y[(size_t)row * U + unit];
                o.tr->yperf[(size_t)it * o.tr->LK + row] = c_sub(yv, make_double2(xa.x / cs, xa.y / cs));
            }
        }
        // a decision exactly on a mid-point (measure zero): the smallest symbol
        // index among the tied grid points (one uniform branch inside)
        slice6(dp, fI, fQ, o.topI, o.topQ, sgrid);
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const bool data = (dmask >> a) & 1;
            ncnt += __umul24(__popc((unsigned)(dp[a] ^ (int)((txp[a >> 2] >> (8 * (a & 3))) & 0xffu))), cweight(a));
            if (TRACE && data && unit == o.tr->unit) o.tr->dec_p[(size_t)it * o.tr->ND + (rdc[4 * a + r] >> 1)] = dp[a];
        }
        if (it < niter) reprecode(dp);                           // the last iteration's decisions are only counted
        cntl[w][it] = wave_sum_dpp(rl < o.rvalid ? ncnt : 0);    // uniform: every lane writes the same word
        ncnt = 0;
    }
    // counters of every stage, summed over the block's 4 waves: thread
    // 2 (it - it0) + edge issues the block's one atomic per counter
    __syncthreads();
    constexpr int it0 = S0 ? 0 : 1;
    if (tid < 2 * (niter + 1 - it0)) {
        const int it = (tid >> 1) + it0, edge = tid & 1;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v += (cntl[k][it] >> (16 * edge)) & 0xffff;
        const int snr = o.snr0 + (ug * WAVE) / R;
        const size_t i0 = o.cidx0 + (size_t)it + (size_t)snr * o.cstride_snr + (edge ? (size_t)o.cstride_edge : 0);
        if (v) atomicAdd(&o.counters[i0], (unsigned long long)v);
    }
}

template <int NT, int SH, bool TRACE, bool S0 = false, bool NM = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_pic_fft(SchemeK sk, BandOrder ord, const double2* __restrict__ ir, int N, StorePerfectDetect o, int niter) {
    pic_fft_body<NT, SH, TRACE, S0, NM>(sk, ord, ir, N, o, niter, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// The MMSE IC iteration of OFDM in structured form (rows a13-a16; k_mic_pilot / k_mic_data below).
// The estimate D_hat = reshape(W hP), W = R_Dij,hP pinv(R) (script:259-313,
// :493-511), is Q' H_hat G: column p of R_Dij,hP is vec(Q' M_p G) with
// M_p = reshape(R_vecH x_p) (script:260), so D_hat = Q' (sum_p M_p z_p) G with
// z = pinv(R) hP, and every M_p lives on the support of the convolution matrix.
// H_hat is therefore a channel estimate with IR's taps,
//   hhat[q][n] = sum_p Bv[q][n][p] hP_p,   Bv = m pinv(R)   (k_bv, m of k_mcoef),
// and y_ic = y - (D_hat - diag D_hat) v (script:482-484) = y - Q'(H_hat (G v)) +
// diag(D_hat) .* v runs as k_pic_fft's DFT-24 chain with the estimated taps.
// For OFDM the 1e-8 thresholds of R_Dij and W (script:264-265, :287-289) only
// drop structural zeros and rounding-level entries (|D_hat - Q' H_hat G| <=
// 4e-11 at C2; dsce_build_mmse verifies diag(D_hat) against the thresholded
// W's diagonal and keeps the contraction otherwise).  diag(D_hat)[l] =
// qs gs sum_q w^(-l d_q) S_q with S_q the sum of hhat[q] over the symbol's FFT
// window: the previous stage's from its taps, this stage's from Bs (window sums
// of Bv) and hP_new.  Per unit and symbol: NT x 24 x NP CMACs for the taps
// instead of the contraction's 24 x 23 x NP.
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// The MMSE branch of an FFT-form OFDM scheme with EVERY stage in one launch
// (r03; rows a13-a16, script:417-537).  The stages of a symbol depend on other
// symbols only through the LS pilot estimates hP_s (script:487-489), and those
// come from the pilot symbols alone: y_ic of a pilot symbol at stage s needs
// only that symbol's stage s - 1 decisions and hP_{s-1}.  So
//   k_mic_pilot: the npb pilot symbols of 16 units per block (one wave per
//                symbol), stages 0..niter; per stage y_ic (stage 0: y), LS at
//                the pilot rows -> hP_s exchanged through LDS (one barrier),
//                diag(D_hat_s) = qs gs sum_q w^(-l d_q) Bs_q hP_s, one-tap,
//                detection, counts; hP_s also to HBM (hpa[s]);
//   k_mic_data:  every other symbol of 64 units per block, stages 0..niter
//                from hpa, the decisions v in registers across the stages.
// Stage s >= 1 of a symbol (either kernel): estimated taps of D_hat_{s-1},
// hhat[q][n] = sum_p Bv(var_{s-1})[q][n][p] hP_{s-1,p} (k_mic_fft's MFMA GEMM,
// 3M), y_ic = y - Q'(H_hat (G v)) + diag(D_hat_{s-1}) v by the DFT-24 chain,
// then the stage's one-tap with diag(D_hat_s) (W up to niter / 2, then W0,
// script:492).  Replaces k_ls + k_stage0_fft (MMSE branch), the pilot pass and
// the niter k_mic_fft launches: y, the transmitted indices and the row tables
// are read once per symbol instead of once per stage, decisions never leave
// the registers, Bv / Bs of both variants are staged once.
// The tap GEMM's A rows interleave the time quarters: tile t row c + 4k is tap
// index 4t + k (q = idx / 6, window sample 6c + idx % 6) of quarter c, so the
// lane quad of a unit pulls its quarter's 4 taps of the tile from one lane with
// ds_bpermute (mic_taps): no LDS slab (k_mic_fft: 52 KB per block; r03's first
// version: a 17 KB per-wave slab with a fence pair per tile).
// ---------------------------------------------------------------------------
struct Mic2Args {
    const double2* __restrict__ bv;   // [var][snr][NT][N][NP]
    const double2* __restrict__ bs;   // [var][snr][nblk][NT][NP]
    double2* hpa;                     // [stage][NP][U]: LS pilot estimates of every stage
    const int* blks;                  // this launch's symbol blocks (k_mic_pilot: the pilot blocks)
    int nb;
    double* mse_err;
    double* mse_pow;
    int nsnr, N, nblk, niter, scheme;
    // low-rank operator (LR): Z = Bz hP per unit and stage, the taps T_k Z
    const double2* bz;                // [var][snr][NT MIC_NB][NP]
    double2* za;                      // [stage][NT MIC_NB][U]
    const double* tw;                 // [nblk][MIC_NB][24]
    const double* ts;                 // [nblk][MIC_NB]
};

__device__ __forceinline__ int mic_var(int s, int niter) { return (s == 0 || 2 * s <= niter) ? 0 : 1; }

// Estimated taps of the lane's six window samples (quad layout: lane r of a unit
// holds samples 6 cq + m) for the 16 units of a wave: MFMA GEMM (3M) with
// A(q, j, p) = Bv[q][klo + j][p] and B = hP (lane (g, jc): pilots 4 ks + g of
// unit jc).  Tile t's A row i is tap index 4 t + (i >> 2) of time quarter i & 3,
// so D register k of lane (g, jc) holds tap index 4 t + k of quarter g, unit jc:
// the lane (unit ul, quarter cq) pulls its four taps of the tile from lane
// 16 cq + ul with one ds_bpermute per dword, the same register in every lane
// (r02-r03's per-wave LDS slab needed 17 KB per block and a fence pair per tile).
// NM (quarters on the 16-lane rows, lane = 16 cq + unit): D register k of a
// lane already is its tap index 4 t + k, no exchange at all.
template <int NT, int NP, bool NM, class ALoad>
__device__ __forceinline__ void mic_taps(double2 (&taps)[6][NT], const ALoad& A, const double2 (&hb)[NP / 4], int l,
                                         int cq) {
    constexpr int NIDX = 6 * NT, NTILE = (NIDX + 3) / 4, NKS = NP / 4;
    const int g = l >> 4, jc = l & 15, ca = jc & 3, ka = jc >> 2, ul = l >> 2;
    const int src = (16 * cq + ul) * 4;
    double br[NKS], bi[NKS], bsm[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        br[ks] = hb[ks].x;
        bi[ks] = hb[ks].y;
        bsm[ks] = hb[ks].x + hb[ks].y;
    }
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
        const int idx = 4 * t + ka;
        const bool ok = (NIDX % 4 == 0) || idx < NIDX;        // compile-time true when the tiles are full
        const int q = idx >= 6 ? 1 : 0, m = idx - 6 * q;
        d4 p1 = d4{0.0, 0.0, 0.0, 0.0}, p2 = p1, p3 = p1;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const double2 a = A(ok ? q : 0, 6 * ca + (ok ? m : 0), 4 * ks + g);
            const double ar = ok ? a.x : 0.0, ai = ok ? a.y : 0.0;
            p1 = MFMA64(ar, br[ks], p1);
            p2 = MFMA64(ai, bi[ks], p2);
            p3 = MFMA64(ar + ai, bsm[ks], p3);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int id2 = 4 * t + k;                     // compile-time
            if (id2 < NIDX) {
                const double2 tv = make_double2(p1[k] - p2[k], p3[k] - p1[k] - p2[k]);
                taps[id2 % 6][id2 / 6] = NM ? tv : bperm_c(src, tv);
            }
        }
    }
}

// x <- qs gs DFT24(sum_q taps_q .* IDFT24(x)(. - d_q)) of one symbol (k_pic_fft's
// chain; twa: the lane twiddles staged in LDS, output scale folded in twa[1])
// NM: k_pic_fft's matrix-core network (amt: A_m per [dir][m][i + 4 k], ai this
// lane's entry; the previous quarter's sample by ds_bpermute)
template <int NT, int SH, bool NM>
__device__ __forceinline__ void mic_chain(double2 (&xx)[6], const double2 (&tp)[6][NT], const double2 (*twa)[4][6],
                                          const double2 (*amt)[6][16], int ai, int l, int r, double sg1, double sg2) {
    dft6<1>(xx);
    double2 t[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        if (NM) {
            t[m] = mfma4_cmul(amt[0][m][ai], xx[p6(m)]);
        } else {
            const double2 p = c_mulf(xx[p6(m)], twa[0][r][m]);
            const double2 pv = dpp_c<QP_XOR2>(p);
            double2 e = make_double2(fma(sg1, p.x, pv.x), fma(sg1, p.y, pv.y));
            e = quad_tw<1>(e, r == 3);
            const double2 qv = dpp_c<QP_XOR1>(e);
            t[m] = make_double2(fma(sg2, e.x, qv.x), fma(sg2, e.y, qv.y));
        }
    }
    const double2 tprev = NM ? bperm_c(((l + 48) & 63) * 4, t[5]) : dpp_c<QP_PREV>(t[5]);
#pragma unroll
    for (int m = 5; m >= 0; --m) {
        const double2 tq = m ? t[m - 1] : tprev;
        double2 acc = make_double2(0.0, 0.0);
#pragma unroll
        for (int q = 0; q < NT; ++q) c_fma(acc, tp[m][q], ((SH >> q) & 1) ? tq : t[m]);
        t[m] = acc;
    }
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        if (NM) {
            xx[m] = mfma4_cmul(amt[1][m][ai], t[m]);
        } else {
            const double2 pv = dpp_c<QP_XOR1>(t[m]);
            double2 f = make_double2(fma(sg2, t[m].x, pv.x), fma(sg2, t[m].y, pv.y));
            f = quad_tw<-1>(f, r == 3);
            const double2 qv = dpp_c<QP_XOR2>(f);
            xx[m] = c_mulf(make_double2(fma(sg1, f.x, qv.x), fma(sg1, f.y, qv.y)), twa[1][r][m]);
        }
    }
    dft6<-1>(xx);
}

// Shared LDS tables of the two kernels: constellation, slicer grid, row tables of
// the wave's symbol, lane twiddles, the per-row diag(D_hat) weight of a delayed tap.
struct Mic2Tables {
    double2 sym[256];
    alignas(16) unsigned char sgrid[256];   // slice6's byte grid [iI][iQ], row stride 16
    double2 twa[2][4][6];
    double2 amt[2][6][16];            // NM network: A_m[i][k] at [dir][m][i + 4 k] (k_pic_fft's)
};

// One-tap + detection of the lane's six rows with diag(D_hat) = hd[a]; returns
// the decided symbol indices (first-minimum tie rule, SignalConstellation.m:88)
__device__ __forceinline__ void mic_detect(int (&dp)[6], const double2 (&ye)[6], const double2 (&hd)[6],
                                           const StorePerfectDetect& o, const unsigned char* sgrid) {
    // z = ye / hd with the slicer scale folded into the reciprocals, and the six
    // rows' 1 / |hd|^2 from ONE reciprocal (r05, batch inversion: prefix
    // products, one recip_fast, two products per row back; 20 FP64 operations
    // instead of 30).  A factor |hd|^2 outside [2^-160, 2^160] (a zero or
    // vanishing estimate somewhere in the lane's rows) takes the per-row
    // reciprocals.
    double nn[6], pp[6], id[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) nn[a] = fma(hd[a].x, hd[a].x, hd[a].y * hd[a].y);
    pp[0] = nn[0];
#pragma unroll
    for (int a = 1; a < 6; ++a) pp[a] = pp[a - 1] * nn[a];
    double inv = recip_fast(pp[5]) * o.scI;                  // scI / prod
#pragma unroll
    for (int a = 5; a > 0; --a) {
        id[a] = inv * pp[a - 1];                              // scI / nn[a]
        inv *= nn[a];
    }
    id[0] = inv;
    // every factor in [2^-160, 2^160] (its exponent field, one unsigned compare
    // per row): then every prefix product stays within 2^(+-960), no denormal
    // (a bound on pp[5] alone let an underflowed prefix through);
    // zero, inf and NaN fail it
    unsigned ex = 0u;
#pragma unroll
    for (int a = 0; a < 6; ++a) ex = max(ex, (unsigned)__double2hiint(nn[a]) - (unsigned)((1023 - 160) << 20));
    const bool ok = ex < (320u << 20);
    if (__ballot(!ok)) {
#pragma unroll
        for (int a = 0; a < 6; ++a) id[a] = ok ? id[a] : recip_fast(nn[a]) * o.scI;
    }
    double fI[6], fQ[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const double2 b = hd[a], y = ye[a];
        const double nx = fma(y.x, b.x, y.y * b.y), ny = fma(y.y, b.x, -(y.x * b.y));
        fI[a] = fma(nx, id[a], o.ofI);
        fQ[a] = fma(ny, id[a] * o.rQ, o.ofQ);
    }
    slice6(dp, fI, fQ, o.topI, o.topQ, sgrid);
}

// The per-unit operands of a symbol, read once (rows 4 a + r): y, the rows'
// constant part of v (precoded pilots / zero rows), transmitted indices; loaded
// by the kernels before their table barrier (r05: after it, the first stage
// waited for them with the barrier's latency behind it)
struct Mic2Unit {
    double2 yv[6], v[6];
    unsigned txp[2];
    __device__ __forceinline__ void load(const StorePerfectDetect& o, int row0, int r, int unit, int rl) {
        const RowView vy(o.y, row0, o.U, r, unit, 16), vx(o.xs, row0, o.R, r, rl, 16), vs(o.sidr, row0, o.R, r, rl, 2);
        txp[0] = txp[1] = 0u;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            yv[a] = vy.ld2(a);
            v[a] = vx.ld2(a);
            txp[a >> 2] |= (vs.ldu16(a) & 0xffu) << (8 * (a & 3));
        }
    }
};

// Stages 0..niter of the MMSE branch for one symbol of a unit (the common body of
// k_mic_pilot and k_mic_data).  PIL: a pilot symbol (LS of every stage into the
// block's LDS exchange + hpa, one barrier per stage); otherwise hP_s comes from
// hpa.  Per-stage counters go to cntl[w][s] (one word per wave and stage).
// LR (the low-rank operator, build_mic_lr): the estimated taps of stage s are
// sum_k T_k[n] Z_{s-1}[q k] with Z_s = Bz(var_s) hP_s (NT MIC_NB values per unit:
// the pilot kernel forms them once per unit and stage, LDS szz + HBM za) and
// T_k the J0 kernel summed over pilot symbol k's window (twl: this symbol's
// window, tsl: its sums), instead of the tap GEMM Bv hP (NT x 24 x NP complex
// MACs per symbol and unit); diag(D_hat_s) from S_q = sum_k tsl[k] Z_s[q k].
template <int NT, int SH, int NP, bool TRACE, bool PIL, bool NM, bool LR, class ALoad, class BsLoad>
__device__ __forceinline__ void mic2_stages(const SchemeK& sk, const Mic2Args& ma, const StorePerfectDetect& o,
                                            const Mic2Unit& mu,
                                            const Mic2Tables& tb, const double2* rpv, const int* rdc, const int* rpc,
                                            const double2* wrow, double2 (*shp)[NP][17],
                                            const double2 (*xpb)[17], int (*cntl), const ALoad& A, const BsLoad& Bs,
                                            int row0, int unit, int unit_mf, int ul, int l, int r, int U, int R, int rl,
                                            int snr, const double* twl = nullptr, const double* tsl = nullptr,
                                            double2 (*szz)[NT * MIC_NB][17] = nullptr, int unit0 = 0,
                                            const double2* bzl = nullptr, double2 (*vcst)[256] = nullptr) {
    constexpr int NZ = NT * MIC_NB;
    const int cq = NM ? r : (r >> 1) + 2 * (r & 1);
    const double sg1 = (r >> 1) ? -1.0 : 1.0, sg2 = (r & 1) ? -1.0 : 1.0;
    const double2 scale = make_double2(o.pf_scale_re, o.pf_scale_im);
    const bool valid = rl < o.rvalid;
    // per-unit operands (mu, loaded by the kernel); PIL: the LS factors isqk / x_p
    // come from the block's LDS table xpb[pilot][unit]
    double2 yv[6], v[6];
    unsigned txp[2] = {mu.txp[0], mu.txp[1]};
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        yv[a] = mu.yv[a];
        v[a] = mu.v[a];
    }
    // this launch's Z of every stage (LR data kernel): [stage][NZ][U] by a buffer view
    const __amdgpu_buffer_rsrc_t rza =
        buf_rsrc(ma.za, LR && !PIL ? (size_t)(ma.niter + 1) * NZ * U * sizeof(double2) : 0);
    unsigned dmask = 0u, emask = 0u;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const int dc = rdc[4 * a + r];
        dmask |= dc >= 0 ? 1u << a : 0u;
        emask |= dc >= 0 && (dc & 1) ? 1u << a : 0u;
    }
    // the data kernel (vcst): the constant rows of v in the lane's own LDS slots
    // (written for every row, read only for the constant ones; no barrier, no
    // other lane reads them), so a re-precoded row is one LDS read behind one
    // address select (k_pic_fft's reprecode, r05)
    if (!PIL)
#pragma unroll
        for (int a = 0; a < 6; ++a) vcst[a][threadIdx.x] = v[a];
    // error-count weight of row a: data rows count 1, no-edge rows also 1 << 16
    auto cweight = [&](int a) -> int {
        return ((dmask >> a) & 1) ? (((emask >> a) & 1) ? 0x10001 : 1) : 0;
    };
    // window sums of the previous stage's estimated taps: diag(D_hat_{s-1}) of the
    // y_ic correction.  They equal Bs hP_{s-1} (Bs = Bv summed over the window),
    // i.e. the previous stage's own diag sums sn, which are kept instead of
    // summing the 12 taps again
    double2 sp0 = make_double2(0.0, 0.0), sp1 = sp0;
    // B operand of the tap GEMM (hP_{s-1}) and this stage's LS pilots (a quarter
    // per lane, for diag(D_hat_s)); the data kernel prefetches both for stage
    // s + 1 at the end of stage s and folds hn4 into the window sums sn at once
    double2 hb[LR ? 1 : NP / 4], hn4[LR ? 1 : NP / 4];
    // LR: Z of this stage (diag, then the next stage's taps), whole unit per lane
    // (the data kernel; the pilot kernel reads them from its LDS szz instead)
    // MLR (r06, the row layout NM): the low-rank taps and window sums on the
    // matrix cores.  MIC_NB = 4 pilot symbols = the K rows of v_mfma_f64_4x4x4f64:
    // the lane of quarter k (row k = l >> 4, unit l & 15 = 4 c + n) holds its
    // unit's Z[q][k] (B[k][n]) and T_k[6 i + a] with i = l & 3 (A[i][k], the same
    // for every block c), so D[i][n] = sum_k T_k[6 i + a] Z_n[q][k] is the tap of
    // sample 6 i + a in the unit's quarter-i lane: 2 MFMAs per (sample, tap)
    // instead of 8 FMAs, and a lane reads 2 of the NZ = 8 Z values per stage
    constexpr bool MLR = LR && NM && MIC_NB == 4;
    constexpr int NZR = LR && !PIL ? (MLR ? NT : NZ) : 1;
    double2 zc[NZR];
    // LR data kernel: the next stage's estimated taps, formed at the end of a stage
    // from its Z (r05: carrying the previous stage's Z instead cost 16 register
    // copies per stage; the taps' live range ends in the chain, so the next
    // stage's land in the same registers)
    constexpr int NTL = LR && !PIL ? 6 : 1;
    double2 ltp[NTL][NT];
    // Z[q][l >> 4] of the lane's unit (MLR)
    auto zrow = [&](int sp, int q) -> double2 { return PIL ? szz[sp & 1][q * MIC_NB + (l >> 4)][ul] : zc[q % NZR]; };
    auto lr_taps = [&](double2 (&tp)[6][NT], int sp, int ozz) {
        if constexpr (MLR) {
            double2 zq[NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) zq[q] = zrow(sp, q);
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double ta = twl[(l >> 4) * 24 + 6 * (l & 3) + a + ozz];
#pragma unroll
                for (int q = 0; q < NT; ++q)
                    tp[a][q] = make_double2(__builtin_amdgcn_mfma_f64_4x4x4f64(ta, zq[q].x, 0.0, 0, 0, 0),
                                            __builtin_amdgcn_mfma_f64_4x4x4f64(ta, zq[q].y, 0.0, 0, 0, 0));
            }
            return;
        }
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            double tk[MIC_NB];
#pragma unroll
            for (int k = 0; k < MIC_NB; ++k) tk[k] = twl[k * 24 + 6 * cq + a + ozz];
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                double2 zk[MIC_NB];
#pragma unroll
                for (int k = 0; k < MIC_NB; ++k)
                    zk[k] = PIL ? szz[sp & 1][q * MIC_NB + k][ul] : zc[(q * MIC_NB + k) % NZR];
                double2 t = make_double2(tk[0] * zk[0].x, tk[0] * zk[0].y);
#pragma unroll
                for (int k = 1; k < MIC_NB; ++k) {
                    t.x = fma(tk[k], zk[k].x, t.x);
                    t.y = fma(tk[k], zk[k].y, t.y);
                }
                tp[a][q] = t;
            }
        }
    };
    // diag(D_hat_s) = qs gs sum_q w^(-l d_q) Bs_q(var_s) hP_s: window sums sn0 / sn1
    auto diag_sums = [&](int s, int ro, double2& sn0, double2& sn1) {
        sn0 = sn1 = make_double2(0.0, 0.0);
        bool f0 = true, f1 = true;                          // compile-time: first tap of each sum assigns
        if constexpr (MLR) {
            const double tsr = tsl[l >> 4];
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                const double2 z = zrow(s, q);
                const double2 sq = make_double2(__builtin_amdgcn_mfma_f64_4x4x4f64(tsr, z.x, 0.0, 0, 0, 0),
                                                __builtin_amdgcn_mfma_f64_4x4x4f64(tsr, z.y, 0.0, 0, 0, 0));
                if ((SH >> q) & 1) {
                    sn1 = f1 ? sq : c_add(sn1, sq);
                    f1 = false;
                } else {
                    sn0 = f0 ? sq : c_add(sn0, sq);
                    f0 = false;
                }
            }
        } else if constexpr (LR) {
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                double2 zk[MIC_NB];
#pragma unroll
                for (int k = 0; k < MIC_NB; ++k) zk[k] = PIL ? szz[s & 1][q * MIC_NB + k][ul] : zc[(q * MIC_NB + k) % NZR];
                double2 sq = make_double2(tsl[0] * zk[0].x, tsl[0] * zk[0].y);
#pragma unroll
                for (int k = 1; k < MIC_NB; ++k) {
                    sq.x = fma(tsl[k], zk[k].x, sq.x);
                    sq.y = fma(tsl[k], zk[k].y, sq.y);
                }
                if ((SH >> q) & 1) {
                    sn1 = f1 ? sq : c_add(sn1, sq);
                    f1 = false;
                } else {
                    sn0 = f0 ? sq : c_add(sn0, sq);
                    f0 = false;
                }
            }
        } else {
            const int vs = mic_var(s, ma.niter);
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                double2 sq = c_mul(Bs(vs, q, ro * (NP / 4)), hn4[0]);
#pragma unroll
                for (int k = 1; k < NP / 4; ++k) c_fma(sq, Bs(vs, q, ro * (NP / 4) + k), hn4[k]);
                if (NM) {
                    // sum over the unit's four quarters (rows): ones(4 x 4) x B
                    sq = make_double2(__builtin_amdgcn_mfma_f64_4x4x4f64(1.0, sq.x, 0.0, 0, 0, 0),
                                      __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, sq.y, 0.0, 0, 0, 0));
                } else {
                    sq = c_add(sq, dpp_c<QP_XOR1>(sq));
                    sq = c_add(sq, dpp_c<QP_XOR2>(sq));
                }
                if ((SH >> q) & 1) {
                    sn1 = f1 ? sq : c_add(sn1, sq);
                    f1 = false;
                } else {
                    sn0 = f0 ? sq : c_add(sn0, sq);
                    f0 = false;
                }
            }
        }
        sn0 = c_mul(scale, sn0);
    };
    for (int s = 0; s <= ma.niter; ++s) {
        // an opaque zero in the per-stage LDS indices: hoisted out of the stage
        // loop, the operator / twiddle reads of both variants would stay live
        // across it (k_pic_fft's lesson)
        int oz = 0;
        asm volatile("" : "+v"(oz));
        const int ro = r + oz;
        double2 sn0, sn1;
        if (MLR && !PIL) {
#pragma unroll
            for (int q = 0; q < NZR; ++q)
                zc[q] = buf_ld2(rza, (unsigned)(unit + (l >> 4) * U) * 16u, (unsigned)((s * NZ + q * MIC_NB) * U) * 16u);
        } else if (LR && !PIL) {
#pragma unroll
            for (int j = 0; j < NZR; ++j) zc[j] = buf_ld2(rza, (unsigned)unit * 16u, (unsigned)((s * NZ + j) * U) * 16u);
        } else if (!LR && !PIL) {
#pragma unroll
            for (int k = 0; k < NP / 4; ++k) hn4[k] = ma.hpa[(size_t)s * NP * U + (size_t)(r * (NP / 4) + k) * U + unit];
        }
        double2 ye[6];
        if (s == 0) {
#pragma unroll
            for (int a = 0; a < 6; ++a) ye[a] = yv[a];
        } else {
            // the previous stage's estimated taps and their window sums
            double2 taps[6][NT];
            if constexpr (LR && !PIL) {
                // formed at the end of stage s - 1 (ltp)
            } else if constexpr (LR) {
                // T_k of the lane's six samples (this symbol's window, quarter cq)
                lr_taps(taps, s - 1, oz);
            } else {
                if (PIL)
#pragma unroll
                    for (int ks = 0; ks < NP / 4; ++ks) hb[ks] = shp[(s - 1) & 1][4 * ks + (l >> 4)][l & 15];
                mic_taps<NT, NP, NM>(taps, [&](int q, int j, int p) { return A(mic_var(s - 1, ma.niter), q, j + oz, p); },
                                     hb, l, cq);
            }
            double2 x[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) x[a] = v[a];
            if constexpr (LR && !PIL)
                mic_chain<NT, SH, NM>(x, ltp, tb.twa, tb.amt, (l & 3) + 4 * (l >> 4) + oz, l, ro, sg1, sg2);
            else
                mic_chain<NT, SH, NM>(x, taps, tb.twa, tb.amt, (l & 3) + 4 * (l >> 4) + oz, l, ro, sg1, sg2);
            // y_ic = y - (D_hat_{s-1} - diag) v  (script:482-484); LR: the taps are
            // mean-free over the window (centred Tw, build_mic_lr), so the chain
            // already is (D_hat - diag) v (r06: 48 FP64 operations per stage fewer)
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                ye[a] = c_sub(yv[a], x[p6(a)]);
                if constexpr (!LR) {
                    double2 hpv = sp0;
                    c_fma(hpv, sp1, wrow[4 * a + ro]);
                    c_fma(ye[a], hpv, v[a]);
                }
            }
        }
        // this stage's LS pilot estimates (script:412-414 / :487-489)
        if (PIL) {
            double2* hx = shp[s & 1][0];
            (void)hx;
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const int pc = rpc[4 * a + r];
                if (pc >= 0) {
                    // xpb holds isqk / x_p (k_mic_pilot's table fill): one product
                    const double2 h = c_mulf(ye[a], xpb[pc][ul]);
                    hx[pc * 17 + ul] = h;
                    if (!LR || TRACE) ma.hpa[((size_t)s * NP + pc) * U + unit] = h;
                }
            }
            __syncthreads();
            if constexpr (LR) {
                // Z_s = Bz(var_s) hP_s for the block's 16 units: one entry per thread
                // (Bz of both variants staged in LDS at kernel start: no global
                // round trip between the stage's two barriers)
                const int vs = mic_var(s, ma.niter);
                const int t = threadIdx.x;
                if (t < NZ * 16) {
                    const int j = t >> 4, u = t & 15;
                    const double2* bz = bzl + ((size_t)vs * NZ + j) * (NP + 1);
                    double2 acc = c_mul(bz[0], hx[u]);
#pragma unroll
                    for (int p = 1; p < NP; ++p) c_fma(acc, bz[p], hx[p * 17 + u]);
                    szz[s & 1][j][u] = acc;
                    ma.za[((size_t)s * NZ + j) * U + unit0 + u] = acc;
                }
                __syncthreads();
            } else {
#pragma unroll
                for (int k = 0; k < NP / 4; ++k) hn4[k] = hx[(r * (NP / 4) + k) * 17 + ul];
            }
            diag_sums(s, ro, sn0, sn1);
        } else {
            diag_sums(s, ro, sn0, sn1);
        }
        double2 hd[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            hd[a] = sn0;
            c_fma(hd[a], sn1, wrow[4 * a + ro]);
        }
        sp0 = sn0;
        sp1 = sn1;
        int dp[6];
        mic_detect(dp, ye, hd, o, tb.sgrid);
        int ncnt = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const bool data = (dmask >> a) & 1;
            ncnt += __umul24(__popc((unsigned)(dp[a] ^ (int)((txp[a >> 2] >> (8 * (a & 3))) & 0xffu))), cweight(a));
            if (TRACE && unit == o.tr->unit) {
                const int row = row0 + 4 * a + r;
                o.tr->yest[(size_t)s * o.tr->LK + row] = ye[a];
                o.tr->hest[(size_t)s * o.tr->LK + row] = hd[a];
                if (data) o.tr->dec_e[(size_t)s * o.tr->ND + (rdc[4 * a + r] >> 1)] = dp[a];
            }
        }
        if (s == ma.niter) {
            // the last stage's decisions are only counted (no re-precoding)
        } else if (PIL) {
            reprecode6(v, dp, dmask, rpv, r, tb.sym, o.pv_uni);
        } else {
            double2 nv[6];
            if (o.pv_uni) {
#pragma unroll
                for (int a = 0; a < 6; ++a) nv[a] = ((dmask >> a) & 1) ? tb.sym[dp[a]] : vcst[a][threadIdx.x];
            } else {
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    const double2 pr = c_mulf(rpv[4 * a + r], tb.sym[dp[a]]), cv = vcst[a][threadIdx.x];
                    nv[a] = ((dmask >> a) & 1) ? pr : cv;
                }
            }
#pragma unroll
            for (int a = 0; a < 6; ++a) v[a] = nv[a];
        }
        cntl[s] = wave_sum_dpp(valid ? ncnt : 0);  // uniform: every lane writes the same word
        if constexpr (LR && !PIL) {
            if (s < ma.niter) {
                int oz2 = 0;
                asm volatile("" : "+v"(oz2));
                lr_taps(ltp, s, oz2);                // stage s + 1's taps from Z_s
            }
        }
        if (!LR && !PIL && s < ma.niter) {
            // stage s + 1's operands: hP_s (tap GEMM) and hP_{s+1} (diag)
            const double2* __restrict__ hs = ma.hpa + (size_t)s * NP * U;
#pragma unroll
            for (int ks = 0; ks < NP / 4; ++ks) hb[ks] = hs[(size_t)(4 * ks + (l >> 4)) * U + unit_mf];
        }
        if (ma.mse_err) {
            double me = 0.0, mp = 0.0;
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double2 hv = o.h[(size_t)(row0 + 4 * a + r) * R + rl];
                const double dx = hd[a].x - hv.x, dy = hd[a].y - hv.y;
                me += dx * dx + dy * dy;
                mp += hv.x * hv.x + hv.y * hv.y;
            }
            flush_mse(me, s == 0 ? mp : 0.0, ma.mse_err, ma.mse_pow, ma.scheme, ma.nsnr, snr, ma.niter + 1, s, valid);
        }
    }
}

// LDS tables of a block: constellation / slicer grid (256 entries), lane twiddles
// Two-phase table staging for 256-thread blocks (r05): mic2_tab_load issues
// every global read of the block tables (one entry of each per thread, clamped,
// unconditional) and of the symbol's row tables (thread rt = min(t, 23)), the
// caller then issues its per-unit reads, and mic2_tab_store writes LDS waiting
// only for the table reads (vmcnt retires in order).  A read under a branch
// waited with vmcnt(0) for everything issued before it.
struct Mic2TabLoad {
    double2 a, tw, t0, pv, wr;
    int rd, pc;
    unsigned g;
};
// r06: the tables come precomputed per scheme (SchemeK::ct_*, build_chain_tables);
// thread tid copies entry tid of each (clamped, unconditional), and thread t the
// row entries of QH block blk (rows row0 .. row0 + 23)
__device__ __forceinline__ void mic2_tab_load(Mic2TabLoad& L, const SchemeK& sk, int blk, int tid, int t) {
    L.a = sk.ct_sym[tid];
    L.g = sk.ct_grid[min(tid, 63)];
    L.tw = sk.ct_twa[min(tid, 47)];
    L.t0 = sk.ct_amt[min(tid, 191)];
    const int i = blk * 24 + min(t, 23);
    L.pv = sk.ct_rpv[i];
    L.rd = sk.ct_rdc[i];
    L.pc = sk.ct_rpc[i];
    L.wr = sk.ct_wrow[i];
}
__device__ __forceinline__ void mic2_tab_store(const Mic2TabLoad& L, Mic2Tables& tb, double2* rpv, int* rdc, int* rpc,
                                               double2* wrow, int tid, int t) {
    tb.sym[tid] = L.a;
    ((unsigned*)tb.sgrid)[min(tid, 63)] = L.g;
    (&tb.twa[0][0][0])[min(tid, 47)] = L.tw;
    (&tb.amt[0][0][0])[min(tid, 191)] = L.t0;
    // row tables (threads t >= 24 rewrite row 23's entries)
    const int rt = min(t, 23);
    rpv[rt] = L.pv;
    rdc[rt] = L.rd;
    rpc[rt] = L.pc;
    wrow[rt] = L.wr;
}

__device__ __forceinline__ void mic2_tables(Mic2Tables& tb, const StorePerfectDetect& o, int tid, int nth) {
    const double2 scale = make_double2(o.pf_scale_re, o.pf_scale_im);
    for (int i = tid; i < 256; i += nth) {
        const double2 a = o.symbols[min(i, o.M - 1)];
        const int gi = i >> 4, gq = i & 15;
        const int g = o.grid_sym[min(gi * o.nQ + gq, o.nI * o.nQ - 1)];
        tb.sym[i] = stage_sym(make_double2(i < o.M ? a.x : 0.0, i < o.M ? a.y : 0.0), o.pv_uni, o.pv_re, o.pv_im);
        tb.sgrid[i] = (unsigned char)(gi < o.nI && gq < o.nQ ? g : 0);
    }
    if (tid < 48) {
        const int e = ((tid / 6) % 4) * (tid % 6);
        const double2 tw = kW24[e % 12];
        const int dir = tid / 24;
        const double2 v = e >= 12 ? make_double2(-tw.x, -tw.y) : tw;
        tb.twa[dir][(tid / 6) % 4][tid % 6] = dir ? c_mul(scale, make_double2(v.x, -v.y)) : v;
    }
    for (int i = tid; i < 192; i += nth) {
        const int dir = i / 96, m = (i / 16) % 6, ii = i & 3, kk = (i >> 2) & 3;
        const int ea = (6 * ii * kk + (dir ? ii : kk) * m) % 24;
        const double2 t0 = kW24[ea % 12];
        const double2 v = ea >= 12 ? make_double2(-t0.x, -t0.y) : t0;
        tb.amt[dir][m][ii + 4 * kk] = dir ? c_mul(scale, make_double2(v.x, -v.y)) : v;
    }
}

// Row tables of symbol block `blk` for the lanes tid < 24 of a wave-group: re-
// precoding value, data index << 1 | no-edge (-1: not a data row), pilot column
// (-1: not a pilot row), diag(D_hat) weight qs gs w^(-l) of a delayed tap
__device__ __forceinline__ void mic2_rows(double2* rpv, int* rdc, int* rpc, double2* wrow, const SchemeK& sk,
                                          const StorePerfectDetect& o, int row0, int t) {
    // clamped, unconditional (threads t >= 24 rewrite row 23's entries): no
    // branch around the reads (r05)
    const int rt = min(t, 23);
    const double2 pv = o.row_pval[row0 + rt];
    const int dr = o.row_data[row0 + rt], cs = o.row_cons[row0 + rt];
    const int pcr = sk.row_pcol[row0 + rt];
    const double2 t0 = kW24[rt % 12];
    rpv[rt] = pv;
    rdc[rt] = dr >= 0 ? (dr << 1) | (cs ? 1 : 0) : -1;
    rpc[rt] = dr < 0 && pcr >= 0 && pcr < sk.NP ? pcr : -1;
    const double2 wl = rt >= 12 ? make_double2(-t0.x, -t0.y) : t0;
    wrow[rt] = c_mul(make_double2(o.pf_scale_re, o.pf_scale_im), make_double2(wl.x, -wl.y));
}

// One wave per pilot symbol (blockDim = 64 npb, npb <= 4), 16 units per block
// (vb / vn: the block index and grid size, as pic_fft_body's)
template <int NT, int SH, int NP, bool TRACE, bool NM, bool LR>
__device__ __forceinline__ void mic_pilot_body(const SchemeK& sk, const Mic2Args& ma, const StorePerfectDetect& o, int vb,
                                               int vn) {
    constexpr int NZ = NT * MIC_NB;
    __shared__ Mic2Tables tb;
    __shared__ double2 rpv[4][24], wrow[4][24];
    __shared__ int rdc[4][24], rpc[4][24];
    __shared__ double2 bss[LR ? 1 : 4][2][NT][NP];          // Bs of each wave's symbol, both variants
    __shared__ double2 shp[2][NP][17];                      // hP of the block's 16 units, double-buffered
    __shared__ double2 xpb[NP][17];                         // isqk / transmitted pilot of the block's 16 units
    __shared__ double2 szz[LR ? 2 : 1][NZ][17];             // LR: Z of the block's 16 units, double-buffered
    __shared__ double twp[LR ? 4 : 1][MIC_NB * 24 + MIC_NB];   // LR: each wave's T_k window + sums
    // LR: Bz of both variants at this SNR, rows padded to NP + 1 (the Z phase's
    // 16-lane groups read rows j and j + 1: unpadded, the same banks; r06,
    // SQ_LDS_BANK_CONFLICT of the pass -33 %)
    __shared__ double2 bzl[LR ? 2 * NZ * (NP + 1) : 1];
    __shared__ int cntl[4][PM_MAXIT + 1];
    const int tid = threadIdx.x, l = tid & 63, r = NM ? l >> 4 : l & 3;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
    const int U = o.U, R = o.R;
    // 16-unit group, SNR-fastest inside each XCD's contiguous range (r05): the
    // SNR points of a realisation share its per-realisation reads (xs, sidr, x_p)
    // in one L2 (unit-major, they sat on different XCDs: 1.72x the algorithmic
    // HBM bytes per launch)
    int ug16;
    {
        const int L = xcd_remap(vb, vn), nch = o.U / o.R;
        ug16 = (L % nch) * (o.R / 16) + L / nch;
    }
    const int ul = NM ? l & 15 : l >> 2;
    const int unit = ug16 * 16 + ul, unit_mf = ug16 * 16 + (l & 15);
    const int rl = unit % R;
    const int snr = o.snr0 + (ug16 * 16) / R;
    const int blk = ma.blks[w];
    const int row0 = sk.QH.row0[blk], klo = sk.QH.klo[blk];
    Mic2Unit mu;
    if (blockDim.x == 256) {
        Mic2TabLoad tl;
        mic2_tab_load(tl, sk, blk, tid, l);
        mu.load(o, row0, r, unit, rl);
        mic2_tab_store(tl, tb, rpv[w], rdc[w], rpc[w], wrow[w], tid, l);
    } else {
        mu.load(o, row0, r, unit, rl);
        mic2_tables(tb, o, tid, blockDim.x);
        mic2_rows(rpv[w], rdc[w], rpc[w], wrow[w], sk, o, row0, l);
    }
    if (LR) {
        for (int i = l; i < MIC_NB * 25; i += 64)
            twp[w][i] = i < MIC_NB * 24 ? ma.tw[(size_t)blk * MIC_NB * 24 + i] : ma.ts[(size_t)blk * MIC_NB + i - MIC_NB * 24];
        for (int i = tid; i < 2 * NZ * NP; i += blockDim.x) {
            const int var = i / (NZ * NP), jp = i % (NZ * NP);
            bzl[(var * NZ + jp / NP) * (NP + 1) + jp % NP] = ma.bz[((size_t)var * ma.nsnr + snr) * NZ * NP + jp];
        }
    } else {
        const int i = min(l, 2 * NT * NP - 1), var = i / (NT * NP), q = (i / NP) % NT, p = i % NP;
        bss[LR ? 0 : w][var][q][p] = ma.bs[(((size_t)(var * ma.nsnr + snr) * ma.nblk + blk) * NT + q) * NP + p];
    }
    // the LS divisor of every pilot of the block's units as isqk / x_p (r05: the
    // per-stage LS of a pilot row is one complex product instead of a division)
    const double isqk0 = sk.inv_sqrt_kappa;
    for (int i = tid; i < NP * 16; i += blockDim.x) {
        const int u16 = ug16 * 16 + (i & 15);
        const double2 xv = o.xp[(size_t)(i >> 4) * R + u16 % R];
        const double id = isqk0 / (xv.x * xv.x + xv.y * xv.y);
        xpb[i >> 4][i & 15] = make_double2(xv.x * id, -xv.y * id);
    }
    __syncthreads();
    const double2* __restrict__ bvb = ma.bv + ((size_t)snr * NT * ma.N + klo) * NP;
    const size_t vstride = (size_t)ma.nsnr * NT * ma.N * NP;
    // the tap GEMM operand straight from L2 (staging each wave's window in LDS,
    // reloaded at the W -> W0 switch: 40 more VGPRs, 1.97 -> 2.28 ms per step)
    auto A = [&](int var, int q, int j, int p) { return bvb[var * vstride + ((size_t)q * ma.N + j) * NP + p]; };
    auto Bs = [&](int var, int q, int p) { return bss[LR ? 0 : w][var][q][p]; };
    mic2_stages<NT, SH, NP, TRACE, true, NM, LR>(sk, ma, o, mu, tb, rpv[w], rdc[w], rpc[w], wrow[w], shp, xpb, cntl[w], A,
                                                 Bs, row0, unit, unit_mf, ul, l, r, U, R, rl, snr, twp[LR ? w : 0],
                                                 twp[LR ? w : 0] + MIC_NB * 24, szz, ug16 * 16, bzl);
    __syncthreads();
    // one atomic per (stage, edge) per block
    for (int i = tid; i < 2 * (ma.niter + 1); i += blockDim.x) {
        const int s = i >> 1, edge = i & 1;
        int v = 0;
        for (int k = 0; k < nw; ++k) v += (cntl[k][s] >> (16 * edge)) & 0xffff;
        const size_t i0 = o.cidx0 + (size_t)s + (size_t)snr * o.cstride_snr + (edge ? (size_t)o.cstride_edge : 0);
        if (v) atomicAdd(&o.counters[i0], (unsigned long long)v);
    }
}

template <int NT, int SH, int NP, bool TRACE, bool NM = false, bool LR = false>
__global__ void __launch_bounds__(256) k_mic_pilot(SchemeK sk, Mic2Args ma, StorePerfectDetect o) {
    mic_pilot_body<NT, SH, NP, TRACE, NM, LR>(sk, ma, o, blockIdx.x, gridDim.x);
}

// 64 units x one data symbol per block (4 waves x 16 units)
template <int NT, int SH, int NP, bool TRACE, bool NM = false, bool LR = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_mic_data(SchemeK sk, BandOrder ord, Mic2Args ma, StorePerfectDetect o) {
    __shared__ Mic2Tables tb;
    __shared__ double2 rpv[24], wrow[24];
    __shared__ int rdc[24], rpc[24];
    constexpr int BVS = NP + 1;
    __shared__ double2 sbv[LR ? 1 : 2][NT][LR ? 1 : 24][BVS];   // Bv of the symbol's window, both variants
    __shared__ double2 bss[2][NT][NP];
    __shared__ double twd[MIC_NB * 24 + MIC_NB];            // LR: T_k over the symbol's window + sums
    __shared__ int cntl[4][PM_MAXIT + 1];
    __shared__ double2 vcst[6][256];                        // each lane's constant rows of v
    int ug, bi;
    band_block(ord, ma.nb, ug, bi);
    const int blk = ma.blks[bi];
    const int tid = threadIdx.x, l = tid & 63, r = NM ? l >> 4 : l & 3;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int U = o.U, R = o.R;
    const int snr = o.snr0 + (ug * WAVE) / R;
    const int ul = NM ? l & 15 : l >> 2;
    const int unit = ug * WAVE + w * 16 + ul, unit_mf = ug * WAVE + w * 16 + (l & 15);
    const int rl = unit % R;
    const int row0 = sk.QH.row0[blk], klo = sk.QH.klo[blk];
    Mic2Unit mu;
    if constexpr (LR) {
        // the load clamped and issued first; only the threads with an entry store
        // (156 threads re-stored entry 99)
        const int i = min(tid, MIC_NB * 25 - 1);
        const double t = i < MIC_NB * 24 ? ma.tw[(size_t)blk * MIC_NB * 24 + i] : ma.ts[(size_t)blk * MIC_NB + i - MIC_NB * 24];
        Mic2TabLoad tl;
        mic2_tab_load(tl, sk, blk, tid, tid);
        mu.load(o, row0, r, unit, rl);
        mic2_tab_store(tl, tb, rpv, rdc, rpc, wrow, tid, tid);
        if (tid < MIC_NB * 25) twd[tid] = t;
    } else {
        // every global load before the first LDS write (clamped, unconditional)
        constexpr int NBV = 2 * NT * 24 * NP, PER = (NBV + 255) / 256;
        double2 bvr[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = min(tid + 256 * k, NBV - 1), var = i / (NT * 24 * NP), q = (i / (24 * NP)) % NT,
                      rem = i % (24 * NP);
            bvr[k] = ma.bv[(((size_t)(var * ma.nsnr + snr) * NT + q) * ma.N + klo) * NP + rem];
        }
        const int ib = min(tid, 2 * NT * NP - 1), var = ib / (NT * NP), q = (ib / NP) % NT, p = ib % NP;
        const double2 bsv = ma.bs[(((size_t)(var * ma.nsnr + snr) * ma.nblk + blk) * NT + q) * NP + p];
        Mic2TabLoad tl;
        mic2_tab_load(tl, sk, blk, tid, tid);
        mu.load(o, row0, r, unit, rl);
        mic2_tab_store(tl, tb, rpv, rdc, rpc, wrow, tid, tid);
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = min(tid + 256 * k, NBV - 1);
            sbv[i / (NT * 24 * NP)][(i / (24 * NP)) % NT][(i / NP) % 24][i % NP] = bvr[k];
        }
        bss[var][q][p] = bsv;
    }
    __syncthreads();
    auto A = [&](int var, int q, int j, int p) { return sbv[LR ? 0 : var][q][LR ? 0 : j][p]; };
    auto Bs = [&](int var, int q, int p) { return bss[var][q][p]; };
    mic2_stages<NT, SH, NP, TRACE, false, NM, LR>(sk, ma, o, mu, tb, rpv, rdc, rpc, wrow, nullptr, nullptr, cntl[w], A, Bs,
                                                  row0, unit, unit_mf, ul, l, r, U, R, rl, snr, twd,
                                                  twd + MIC_NB * 24, nullptr, 0, nullptr, vcst);
    __syncthreads();
    for (int i = tid; i < 2 * (ma.niter + 1); i += 256) {
        const int s = i >> 1, edge = i & 1;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v += (cntl[k][s] >> (16 * edge)) & 0xffff;
        const size_t i0 = o.cidx0 + (size_t)s + (size_t)snr * o.cstride_snr + (edge ? (size_t)o.cstride_edge : 0);
        if (v) atomicAdd(&o.counters[i0], (unsigned long long)v);
    }
}

// ---------------------------------------------------------------------------
// TX, channel and receiver front of an FFT-form OFDM scheme in one pass
// (k_txrx_fft, rows a7, a8, a12; script:371-409): per realisation and symbol
// s = gs IDFT24(x) (G with its cyclic prefix), r0[n] = sum_q IR_q[n] s[n - d_q]
// (GetConvolutionMatrix, FastFading.m:284), and for every SNR point of the
// chunk y = qs DFT24(r0 + sqrt(Pn/2) z) with z the noise stream of LoadNoisy
// (identical draws); the perfect-CSI diag(D) = qs gs sum_q w^(-l d_q) S_q(IR)
// (S_q = the window sum of tap q).  Replaces the G band, k_channel_apply, the
// diag(D) band and the noisy Q^H band: s and r0 never reach memory.  A
// realisation's four time quarters sit on the four 16-lane rows (lane = 16 r +
// realisation, k_pic_fft's NM layout), block = 64 realisations x one symbol; the
// 4-point network of both transforms is one complex 4 x 4 product per sample
// on the matrix cores (r05: the DPP network cost 100 cycles per sample and
// wave against 72, and the quad sums of diag(D) are one ones-MFMA each).
// ---------------------------------------------------------------------------
constexpr int TXRX_MAXSNR = 64;      // SNR points per k_txrx_fft launch (the launcher checks)

struct TxrxArgs {
    const double2* __restrict__ xs;   // [LK][R] precoded symbols P [xP; xD]
    const double2* __restrict__ ir;   // [ntap][N][R]
    const double* __restrict__ pn;    // [nsnr]
    double2* y;                       // [LK][U]
    double2* h;                       // [LK][R]
    uint64_t seed, rep0;
    int N, R, U, snr0, nchunk, slot, base;
};

template <int NT, int SH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_txrx_fft(SchemeK sk, TxrxArgs ta, int xcd) {
    // block: 64 realisations x one symbol, XCD-aware (symbol fastest)
    int L = blockIdx.x;
    if (xcd) L = xcd_remap(L, gridDim.x);
    const int blk = L % sk.QH.nblk, rg = L / sk.QH.nblk;
    const int tid = threadIdx.x, l = tid & 63, r = l >> 4, w = tid >> 6;
    const int rl = rg * WAVE + w * 16 + (l & 15);
    const int R = ta.R;
    const int cq = r;                                           // time quarter of this lane
    const int row0 = sk.QH.row0[blk], klo = sk.QH.klo[blk];
    __shared__ double2 amt[2][6][16];                          // A_m[i][k] at [dir][m][i + 4 k]
    __shared__ double2 wrow[24];
    __shared__ double ssc[TXRX_MAXSNR];                        // sqrt(Pn / 2) of the chunk's SNR points
    __shared__ double2 slt[128], sct[256];                     // the Box-Muller tables (bm_tables.h)
    const double2 gs = sk.pf_gs, qs = sk.pf_qs, ps = sk.pf_scale;
    double2 x[6], taps[6][NT];
    {
        // table loads (twiddles, noise powers), then the per-unit loads, then
        // the LDS writes (unconditional, clamped: a write under a branch lets
        // the compiler sink its load there, behind a vmcnt(0))
        // A_m[i][k]: inverse gs w24^(6 i k + k m), forward qs w24^-(6 i k + i m)
        const int tc = min(tid, 191);
        const int dir = tc / 96, mm = (tc / 16) % 6, ii = tc & 3, kk = (tc >> 2) & 3;
        const int ea = (6 * ii * kk + (dir ? ii : kk) * mm) % 24;
        const double2 tw = kW24[ea % 12];
        const int lr0 = min(max(tid - 64, 0), 23);
        const double2 t0 = kW24[lr0 % 12];
        const int kc = min(tid, ta.nchunk - 1);
        const double pnv = ta.pn[ta.snr0 + kc];
        const double2 cv = kCisT[tid], lv = kLogT[tid & 127];
#pragma unroll
        for (int a = 0; a < 6; ++a) x[a] = ta.xs[(size_t)(row0 + 4 * a + r) * R + rl];
#pragma unroll
        for (int m = 0; m < 6; ++m)
#pragma unroll
            for (int q = 0; q < NT; ++q) taps[m][q] = ta.ir[((size_t)q * ta.N + klo + 6 * cq + m) * R + rl];
        const double2 v = ea >= 12 ? make_double2(-tw.x, -tw.y) : tw;
        amt[dir][mm][ii + 4 * kk] = dir ? c_mul(qs, make_double2(v.x, -v.y)) : c_mul(gs, v);
        const double2 wl = lr0 >= 12 ? make_double2(-t0.x, -t0.y) : t0;
        wrow[lr0] = c_mul(ps, make_double2(wl.x, -wl.y));
        ssc[kc] = sqrt(pnv / 2.0);
        sct[tid] = cv;
        slt[tid & 127] = lv;
    }
    __syncthreads();
    const int ai = (l & 3) + 4 * (l >> 4);                    // this lane's A entry
    // perfect-CSI diag(D) of the symbol's rows from the window sums of the taps
    {
        double2 s0 = make_double2(0.0, 0.0), s1 = s0;
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            double2 sq = make_double2(0.0, 0.0);
#pragma unroll
            for (int m = 0; m < 6; ++m) sq = c_add(sq, taps[m][q]);
            // sum over the realisation's four quarters (rows): ones(4 x 4) x B
            sq = make_double2(__builtin_amdgcn_mfma_f64_4x4x4f64(1.0, sq.x, 0.0, 0, 0, 0),
                              __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, sq.y, 0.0, 0, 0, 0));
            if ((SH >> q) & 1) s1 = c_add(s1, sq);
            else s0 = c_add(s0, sq);
        }
        s0 = c_mul(ps, s0);
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            double2 hv = s0;
            c_fma(hv, s1, wrow[4 * a + r]);
            if (ta.snr0 == 0) ta.h[(size_t)(row0 + 4 * a + r) * R + rl] = hv;
        }
    }
    // s = gs IDFT24(x): lane r ends with the time samples 6 cq + m
    dft6<1>(x);
    double2 t[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) t[m] = mfma4_cmul(amt[0][m][ai], x[p6(m)]);
    // r0 = H s over the window (the delayed tap reads the cyclic prefix for m = 0
    // of quarter 0: sample 5 of quarter 3)
    double2 r0[6];
    {
        const double2 tprev = bperm_c(((l + 48) & 63) * 4, t[5]);
#pragma unroll
        for (int m = 5; m >= 0; --m) {
            const double2 tp = m ? t[m - 1] : tprev;
            double2 acc = make_double2(0.0, 0.0);
#pragma unroll
            for (int q = 0; q < NT; ++q) c_fma(acc, taps[m][q], ((SH >> q) & 1) ? tp : t[m]);
            r0[m] = acc;
        }
    }
    // per SNR point: r = r0 + noise (LoadNoisy's draws), y = qs DFT24(r); the
    // first Philox round of every sample is SNR-independent (stream_pre)
    PhiloxSub phs[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) phs[m] = stream_pre(ta.seed, ta.rep0 + (uint64_t)rl, (uint32_t)(klo + 6 * cq + m));
    for (int k = 0; k < ta.nchunk; ++k) {
        const int snr = ta.snr0 + k;
        const double sc = ssc[k];
        double2 f[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            const uint4 wr = stream_sub(phs[m], STREAM_NOISE, (uint32_t)(ta.base + snr + 256 * ta.slot));
            f[m] = mfma4_cmul(amt[1][m][ai], noise_add(r0[m], sc, wr, slt, sct));
        }
        dft6<-1>(f);
        const size_t u0 = (size_t)k * R + rl;
#pragma unroll
        for (int a = 0; a < 6; ++a) ta.y[(size_t)(row0 + 4 * a + r) * ta.U + u0] = f[p6(a)];
    }
}

bool txrx_fft_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b);

template <int NT, class Out>
static void launch_pass2(hipStream_t s, const SchemeK& sk, const ChannelK& ch, McBuffers& b, const BandOrder& ord,
                         const Out& o, size_t lds) {
    LoadChannelApplied<NT> in{};
    in.t = b.t;
    in.ir = b.ir;
    in.U = b.U;
    in.R = b.R;
    in.N = ch.N;
    in.ntap = ch.ntap;
    for (int q = 0; q < ch.ntap && q < (NT > 0 ? NT : DSCE_MAX_TAPS); ++q) in.delay[q] = ch.tap_delay[q];
    launch_band(s, sk.QH, b.U, &ord, in, o, lds);
}

template <class Out>
static void launch_pass2_nt(hipStream_t s, const SchemeK& sk, const ChannelK& ch, McBuffers& b, const BandOrder& ord,
                            const Out& o, size_t lds = 0) {
    switch (ch.ntap) {
        case 1: launch_pass2<1>(s, sk, ch, b, ord, o, lds); break;
        case 2: launch_pass2<2>(s, sk, ch, b, ord, o, lds); break;
        case 3: launch_pass2<3>(s, sk, ch, b, ord, o, lds); break;
        case 4: launch_pass2<4>(s, sk, ch, b, ord, o, lds); break;
        case 5: launch_pass2<5>(s, sk, ch, b, ord, o, lds); break;
        case 6: launch_pass2<6>(s, sk, ch, b, ord, o, lds); break;
        default: launch_pass2<0>(s, sk, ch, b, ord, o, lds); break;
    }
}

// Opts::pic_chain: 0 = per-iteration passes (G u pass + Q^H H pass), 3 (default)
// = k_pic_fft where the scheme allows it, else the passes.
// k_pic_fft's SH for the channel's taps (-1: no instance): delays <= 1
static int pic_fft_shift(const ChannelK& ch) {
    if (ch.ntap < 1 || ch.ntap > 2) return -1;
    int sh = 0;
    for (int q = 0; q < ch.ntap; ++q) {
        if (ch.tap_delay[q] > 1) return -1;
        sh |= ch.tap_delay[q] << q;
    }
    return (ch.ntap == 1 && sh == 0) || (ch.ntap == 2 && (sh == 1 || sh == 2)) ? sh : -1;
}

// k_txrx_fft applies: FFT-form OFDM blocks, at most two taps with delays <= 1,
// every sample of the scheme's frame read by exactly one Q^H block
bool txrx_fft_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b) {
    return op.txrx_fft && op.noise_fuse && sk.pf_ok && sk.qh_disjoint && pic_fft_shift(ch) >= 0 &&
           (b.R % WAVE) == 0 && b.U / b.R <= TXRX_MAXSNR && (long long)ch.ntap * ch.N * b.R < (1ll << 40);
}

static unsigned launch_txrx(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, const double* pn,
                            uint64_t seed, uint64_t rep0, McBuffers& b) {
    TxrxArgs ta{};
    ta.xs = b.xs;
    ta.ir = b.ir;
    ta.pn = pn;
    ta.y = b.y;
    ta.h = b.h;
    ta.seed = seed;
    ta.rep0 = rep0;
    ta.N = ch.N;
    ta.R = b.R;
    ta.U = b.U;
    ta.snr0 = b.snr0;
    ta.nchunk = b.U / b.R;
    ta.slot = sk.noise_slot;
    ta.base = op.snr_base;
    const dim3 grid((b.R / WAVE) * sk.QH.nblk), blk(256);
    if (ch.ntap == 1) hipLaunchKernelGGL((k_txrx_fft<1, 0>), grid, blk, 0, s, sk, ta, op.xcd);
    else if (pic_fft_shift(ch) == 1) hipLaunchKernelGGL((k_txrx_fft<2, 1>), grid, blk, 0, s, sk, ta, op.xcd);
    else hipLaunchKernelGGL((k_txrx_fft<2, 2>), grid, blk, 0, s, sk, ta, op.xcd);
    return PATH_NOISE_FUSED | PATH_TXRX_FFT;
}

static bool pic_fft_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b, int niter) {
    const bool fits = (long long)24 * b.U * 16 < (1ll << 32) && (long long)ch.ntap * ch.N * b.R * 16 < (1ll << 32) &&
                      (long long)sk.LK * b.U < (1ll << 62);
    // slice6's byte grid: nI, nQ <= 16 levels, M <= 256 symbols
    return sk.pf_ok && op.pic_chain == 3 && pic_fft_shift(ch) >= 0 && fits && niter >= 1 && niter <= PM_MAXIT &&
           sk.M <= 256 && sk.nI <= 16 && sk.nQ <= 16;
}

bool perfect_chain_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b, int niter) {
    return pic_fft_ok(op, sk, ch, b, niter);
}

// Detection operands of the chain kernels (k_pic_fft / k_mic_pilot /
// k_mic_data): tables, slicer folded for nearest_lin, counters of branch `csi`
// (0 MMSE, 1 perfect CSI; the stage is added per iteration).
static StorePerfectDetect chain_detect(const SchemeK& sk, const McBuffers& b, const PerfectDetectArgs* pd, int csi) {
    StorePerfectDetect o{};
    o.tr = b.tr;
    o.y = b.y;
    o.h = b.h;
    o.u = b.u;
    o.sidx = b.sidx;
    o.row_data = sk.row_data;
    o.row_cons = sk.row_cons;
    o.row_pval = sk.row_pval;
    o.symbols = sk.symbols;
    o.lvI = sk.lvI;
    o.lvQ = sk.lvQ;
    o.grid_sym = sk.grid_sym;
    o.counters = pd->counters;
    o.cidx0 = ((((size_t)pd->scheme * 2 + csi) * 2 + 0) * pd->nsnr) * pd->nstage;
    o.cstride_edge = pd->nsnr * pd->nstage;
    o.cstride_snr = pd->nstage;
    o.U = b.U;
    o.R = b.R;
    o.rvalid = b.rvalid;
    o.snr0 = b.snr0;
    o.M = sk.M;
    o.nI = sk.nI;
    o.nQ = sk.nQ;
    o.real_detect = sk.real_detect;
    o.idd = 1.0 / sk.data_div;
    o.sI = pd->sI;
    o.sQ = pd->sQ;
    o.xp = b.xp;
    o.xs = b.xs;
    o.sidr = b.sidr;
    o.scI = o.idd * o.sI;
    o.ofI = 0.5 - sk.lv0I * o.sI;
    o.topI = sk.nI - 1;
    o.scQ = sk.real_detect ? 0.0 : o.idd * o.sQ;
    o.ofQ = 0.5 - sk.lv0Q * o.sQ;
    o.topQ = sk.nQ - 1;
    o.rQ = o.scI != 0.0 ? o.scQ / o.scI : 0.0;
    o.pf_scale_re = sk.pf_scale.x;
    o.pf_scale_im = sk.pf_scale.y;
    o.pv_uni = sk.pv_uni;
    o.pv_re = sk.pv_data.x;
    o.pv_im = sk.pv_data.y;
    return o;
}

// Every stage of the MMSE branch of an FFT-form OFDM scheme (k_mic_pilot over the
// pilot symbols, then k_mic_data over the others; see Mic2Args).
bool mmse_stages_ok(const Opts& op, const SchemeK& sk, const MmseK& mm, const ChannelK& ch, const McBuffers& b,
                    int niter) {
    // (the data kernel's buffer view of Z: every stage's NT MIC_NB x U entries < 4 GB)
    const bool fits = (long long)ch.ntap * ch.N * 16 < (1ll << 31) && (long long)sk.LK * b.U < (1ll << 62) &&
                      (long long)(niter + 1) * 2 * MIC_NB * b.U * 16 < (1ll << 32);
    return op.mmse_ic == 1 && mm.Bv && mm.Bs && sk.pf_ok && sk.NP == 16 && pic_fft_shift(ch) >= 0 &&
           (b.U % 64) == 0 && (b.R % 64) == 0 && fits && mm.npb >= 1 && mm.npb <= 4 && mm.ndb >= 1 && b.hpa &&
           niter >= 1 && niter <= PM_MAXIT && b.hpa_stages >= niter + 1 && op.pic_chain == 3 &&
           pic_fft_ok(op, sk, ch, b, niter) && (long long)(niter + 1) * sk.NP * b.U < (1ll << 40);
}

static Mic2Args mic2_args(const SchemeK& sk, const MmseK& mm, const ChannelK& ch, const McBuffers& b,
                          const PerfectDetectArgs* pd, int niter) {
    Mic2Args ma{};
    ma.bv = mm.Bv;
    ma.bs = mm.Bs;
    ma.hpa = b.hpa;
    ma.mse_err = b.mse_err;
    ma.mse_pow = b.mse_pow;
    ma.nsnr = mm.nsnr;
    ma.N = ch.N;
    ma.nblk = sk.QH.nblk;
    ma.niter = niter;
    ma.scheme = pd->scheme;
    ma.bz = mm.Bz;
    ma.za = b.za;
    ma.tw = mm.Tw;
    ma.ts = mm.Ts;
    ma.blks = mm.pblk;
    ma.nb = mm.npb;
    return ma;
}

unsigned launch_mmse_stages(hipStream_t s, const SchemeK& sk, const MmseK& mm, const ChannelK& ch, McBuffers& b,
                            const PerfectDetectArgs* pd, int niter, int xcd, int part, bool nm, bool lr) {
    StorePerfectDetect o = chain_detect(sk, b, pd, 0);
    Mic2Args ma = mic2_args(sk, mm, ch, b, pd, niter);
    // the low-rank operator: built (build_mic_lr), MIC_NB pilot symbols, Z buffer;
    // the data pass on the matrix-core network (the caller requires mic_net bit 0)
    const bool use_lr = lr && mm.Bz && mm.Tw && mm.Ts && b.za && mm.npb == MIC_NB;
    const int sh = pic_fft_shift(ch);
    // pilot symbols: one wave each, 16 units per block
    ma.blks = mm.pblk;
    ma.nb = mm.npb;
    if (part & 1) {
        const dim3 grid(b.U / 16), blk(64 * mm.npb);
        const bool pnm = nm;
#define LAUNCH_MP(NTV, SHV)                                                                                  \
    do {                                                                                                     \
        if (use_lr && b.tr && pnm) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, true, true, true>), grid, blk, 0, s, sk, ma, o); \
        else if (use_lr && pnm) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, false, true, true>), grid, blk, 0, s, sk, ma, o); \
        else if (use_lr && b.tr) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, true, false, true>), grid, blk, 0, s, sk, ma, o); \
        else if (use_lr) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, false, false, true>), grid, blk, 0, s, sk, ma, o); \
        else if (b.tr && pnm) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, true, true>), grid, blk, 0, s, sk, ma, o); \
        else if (b.tr) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, true>), grid, blk, 0, s, sk, ma, o);   \
        else if (pnm) hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, false, true>), grid, blk, 0, s, sk, ma, o); \
        else hipLaunchKernelGGL((k_mic_pilot<NTV, SHV, 16, false>), grid, blk, 0, s, sk, ma, o);            \
    } while (0)
        if (ch.ntap == 1) LAUNCH_MP(1, 0);
        else if (sh == 1) LAUNCH_MP(2, 1);
        else LAUNCH_MP(2, 2);
#undef LAUNCH_MP
    }
    ma.blks = mm.dblk;
    ma.nb = mm.ndb;
    if (part & 2) {
        const BandOrder om{b.U / WAVE, b.U / b.R, b.R / WAVE, xcd};
        const dim3 grid((b.U / WAVE) * mm.ndb), blk(256);
        const bool dlr = use_lr && nm;
#define LAUNCH_MD(NTV, SHV)                                                                                  \
    do {                                                                                                     \
        if (dlr && b.tr) hipLaunchKernelGGL((k_mic_data<NTV, SHV, 16, true, true, true>), grid, blk, 0, s, sk, om, ma, o); \
        else if (dlr) hipLaunchKernelGGL((k_mic_data<NTV, SHV, 16, false, true, true>), grid, blk, 0, s, sk, om, ma, o); \
        else if (b.tr && nm) hipLaunchKernelGGL((k_mic_data<NTV, SHV, 16, true, true>), grid, blk, 0, s, sk, om, ma, o); \
        else if (b.tr) hipLaunchKernelGGL((k_mic_data<NTV, SHV, 16, true>), grid, blk, 0, s, sk, om, ma, o); \
        else if (nm) hipLaunchKernelGGL((k_mic_data<NTV, SHV, 16, false, true>), grid, blk, 0, s, sk, om, ma, o); \
        else hipLaunchKernelGGL((k_mic_data<NTV, SHV, 16, false>), grid, blk, 0, s, sk, om, ma, o);         \
    } while (0)
        if (use_lr && !dlr)
            throw std::logic_error("launch_mmse_stages: the low-rank pilot pass needs the low-rank data pass "
                                   "(mic_net bit 0)");
        if (ch.ntap == 1) LAUNCH_MD(1, 0);
        else if (sh == 1) LAUNCH_MD(2, 1);
        else LAUNCH_MD(2, 2);
#undef LAUNCH_MD
    }
    return PATH_MIC_FFT | PATH_MIC_STAGES | (use_lr ? PATH_MIC_LR : 0u);
}

unsigned launch_perfect_chain(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, McBuffers& b,
                              const PerfectDetectArgs* pd, int niter, bool stage0) {
    if (!pic_fft_ok(op, sk, ch, b, niter))
        throw std::logic_error("launch_perfect_chain: no chain kernel for this scheme (perfect_chain_ok is false)");
    StorePerfectDetect o = chain_detect(sk, b, pd, 1);
    const BandOrder om{b.U / WAVE, b.U / b.R, b.R / WAVE, op.xcd};
    const dim3 grid((b.U / WAVE) * sk.QH.nblk), blk(256);
    // stage0: the chain also runs stage 0 of the branch (with k_mic_pilot /
    // k_mic_data); otherwise stage 0 came from the stage kernel (u in HBM)
    if (!(o.scI != 0.0))
        throw std::logic_error("launch_perfect_chain: the chain's slicer scale is zero");
#define LAUNCH_PF(NTV, SHV, S0V, NMV)                                                                               \
    do {                                                                                                             \
        if (b.tr)                                                                                                    \
            hipLaunchKernelGGL((k_pic_fft<NTV, SHV, true, S0V, NMV>), grid, blk, 0, s, sk, om, b.ir, ch.N, o, niter);  \
        else                                                                                                         \
            hipLaunchKernelGGL((k_pic_fft<NTV, SHV, false, S0V, NMV>), grid, blk, 0, s, sk, om, b.ir, ch.N, o, niter); \
    } while (0)
    // Opts::pic_net: the 4-point network on the matrix cores (1) or by DPP (0)
#define LAUNCH_PF2(NTV, SHV)                              \
    do {                                                  \
        if (stage0 && op.pic_net) LAUNCH_PF(NTV, SHV, true, true);    \
        else if (stage0) LAUNCH_PF(NTV, SHV, true, false);            \
        else if (op.pic_net) LAUNCH_PF(NTV, SHV, false, true);        \
        else LAUNCH_PF(NTV, SHV, false, false);                       \
    } while (0)
    const int sh = pic_fft_shift(ch);
    if (ch.ntap == 1) LAUNCH_PF2(1, 0);
    else if (sh == 1) LAUNCH_PF2(2, 1);
    else LAUNCH_PF2(2, 2);
#undef LAUNCH_PF2
#undef LAUNCH_PF
    return PATH_PIC_FFT;
}

// ---------------------------------------------------------------------------
// Perfect-CSI IC of polyphase schemes (SchemeK::poly_ok, build_poly in
// dsce_api.hip): D u = Q^H H G u (script:541-543) without the two banded passes.
// Every column of symbol k of G is a real window times a subcarrier tone,
// G[n, l + L k] = A_k[n] w^(l n) C[l][k] (FBMC: the Hermite prototype shifted by
// k TimeSpacing, FBMC.m:255-285 / :318-354; w = e^(2 pi i / F), F = L), so
//   t = G u:      t[n] = sum_k A_k[n] V_k[n mod F],  V_k = IDFT_F(C_k u_k)
//   r0 = H t:     r0[n] = sum_q IR_q[n] t[n - d_q]  (FastFading.m:284)
//   Q^H r0:       out[l + L k] = E[l][k] DFT_F(fold_k)[l],
//                 fold_k[m] = sum_{n = m mod F} B_k[n] r0[n]
// FBMC at C3 (F = 24, 30 symbols, windows of 192 samples): 2 x 30 DFT-24 and
// 2 x 540 x 16 window products per unit instead of 2 x 138 k complex MACs.
// k_poly_syn (symbol-major) writes V, k_poly_chan (residue-major: the samples
// n = m + F j of one residue m are one register array) writes fold, k_poly_ana
// (symbol-major) transforms and hands each row to the pass-2 epilogue (Out:
// StorePerfectIC, or StorePerfectDetect for row-local precoders).  Lane = unit.
// ---------------------------------------------------------------------------
struct PolyArgs {
    const double2* __restrict__ u;    // [LK][U]
    double2* __restrict__ v;          // [LK][U]  V_k[m] at row k F + m
    double2* __restrict__ fo;         // [LK][U]  fold_k[m] at row k F + m, samples of the first half
    double2* __restrict__ fo2;        // [LK][U]  ... of the second half
    const double2* __restrict__ C;    // [K][F]
    const double2* __restrict__ E;    // [K][F]
    const double* __restrict__ A;     // [F][K][POLY_NA]: A(j) at j + 1, index 0 = 0
    const double* __restrict__ B;     // [F][K][POLY_NI]
    const double2* __restrict__ tw;   // w^e, e = 0..F-1
    const double2* __restrict__ ir;   // [ntap][N][R]
    int U, R, K, N, xcd;
    int delay[4];
};

// x * w^(S e) (e a compile-time exponent after unrolling: the table entry is a
// uniform load, and e = 0 mod F costs nothing)
template <int F, int S>
__device__ __forceinline__ double2 poly_tw(double2 x, int e, const double2* __restrict__ tw) {
    const int i = ((S * e) % F + F) % F;
    if (i == 0) return x;
    return c_mulf(x, tw[i]);
}

// y[m] = sum_l x[l] w^(S l m), F = 3 F2: DFT-3 over l1 (l = F2 l1 + l2), twiddle
// w^(S l2 m1), then a DFT-F2 over l2 per m1 (m = m1 + 3 m2), each output handed
// to emit(m, y[m]) as soon as it is formed.  x is overwritten.
template <int F, int S, class Emit>
__device__ __forceinline__ void poly_dft(double2 (&x)[F], const double2* __restrict__ tw, Emit&& emit) {
    static_assert(F % 3 == 0, "F = 3 F2");
    constexpr int F2 = F / 3;
    constexpr double H3 = 0.86602540378443864676;   // sqrt(3) / 2
#pragma unroll
    for (int l2 = 0; l2 < F2; ++l2) {
        const double2 x0 = x[l2], x1 = x[F2 + l2], x2 = x[2 * F2 + l2];
        const double2 sm = c_add(x1, x2), df = c_sub(x1, x2);
        const double2 mm = make_double2(fma(-0.5, sm.x, x0.x), fma(-0.5, sm.y, x0.y));
        const double2 jd = make_double2(-S * H3 * df.y, S * H3 * df.x);   // j S (sqrt 3 / 2) (x1 - x2)
        x[l2] = c_add(x0, sm);
        x[F2 + l2] = poly_tw<F, S>(c_add(mm, jd), l2, tw);
        x[2 * F2 + l2] = poly_tw<F, S>(c_sub(mm, jd), 2 * l2, tw);
    }
#pragma unroll
    for (int m1 = 0; m1 < 3; ++m1)
#pragma unroll
        for (int m2 = 0; m2 < F2; ++m2) {
            double2 acc = x[F2 * m1];
#pragma unroll
            for (int l2 = 1; l2 < F2; ++l2) {
                const int i = ((S * 3 * l2 * m2) % F + F) % F;
                if (i == 0) acc = c_add(acc, x[F2 * m1 + l2]);
                else c_fma(acc, x[F2 * m1 + l2], tw[i]);
            }
            emit(m1 + 3 * m2, acc);
        }
}

// block -> (unit group, index) with the index fastest, XCD-aware
__device__ __forceinline__ void poly_block(int nidx, int xcd, int& ug, int& idx) {
    int L = blockIdx.x;
    if (xcd) L = xcd_remap(L, gridDim.x);
    idx = L % nidx;
    ug = L / nidx;
}

template <int F>
__global__ void __launch_bounds__(64) k_poly_syn(PolyArgs pa) {
    int ug, k;
    poly_block(pa.K, pa.xcd, ug, k);
    const int lane = ug * WAVE + threadIdx.x;
    const double2* __restrict__ cg = pa.C + (size_t)k * F;
    double2 x[F];
#pragma unroll
    for (int l = 0; l < F; ++l) x[l] = c_mulf(cg[l], pa.u[(size_t)(k * F + l) * pa.U + lane]);
    double2* __restrict__ out = pa.v + (size_t)k * F * pa.U + lane;
    poly_dft<F, 1>(x, pa.tw, [&](int m, double2 y) { out[(size_t)m * pa.U] = y; });
}

// Block = (unit group, residue m, half h): the half's POLY_IH samples
// n = m + F i, i in [h IH, (h + 1) IH), and its partial window sums into fo
// (h = 0) / fo2 (h = 1), which k_poly_ana adds.  Halves keep a wave at ~150
// VGPRs (3 waves per SIMD) where the whole residue (r0 and t of 24 samples)
// took 288 and one wave per SIMD left the V loads' latency exposed (r04 box,
// C3: 6.3 -> 3.6 ms per iteration; the two halves as the waves of one block,
// their partial sums met in LDS instead of fo2: 5.3 ms, LDS-limited occupancy
// and the barrier cost more than the extra 16 B per entry).
template <int F, int NT>
__global__ void __launch_bounds__(64) k_poly_chan(PolyArgs pa) {
    int ug, mh;
    poly_block(2 * F, pa.xcd, ug, mh);
    const int m = mh >> 1, h = mh & 1, i0 = h * POLY_IH;
    const int lane = ug * WAVE + threadIdx.x, rep = lane % pa.R;
    double2 r0[POLY_IH];
#pragma unroll
    for (int i = 0; i < POLY_IH; ++i) r0[i] = make_double2(0.0, 0.0);
#pragma unroll
    for (int q = 0; q < NT; ++q) {
        // t at the samples mq + F j, j = i0 - 1 + jj (jj = 0..IH): the tap's
        // n - d_q = mq + F (i - sh) for the half's r0[i]
        int mq = m - pa.delay[q], sh = 0;
        if (mq < 0) {
            mq += F;
            sh = 1;
        }
        double2 t[POLY_IH + 1];
#pragma unroll
        for (int j = 0; j <= POLY_IH; ++j) t[j] = make_double2(0.0, 0.0);
        const double2* __restrict__ vq = pa.v + (size_t)mq * pa.U + lane;
        // A(j) at index j + 1 (index 0: j = -1, zero): the half's t[jj] reads index i0 + jj
        const double* __restrict__ aq = pa.A + (size_t)mq * pa.K * POLY_NA + i0;
        // V_k[mq] in groups of PG symbols, the next group requested before the
        // current one's products
        constexpr int PG = 4;
        double2 vb[PG];
#pragma unroll
        for (int g = 0; g < PG; ++g) vb[g] = vq[(size_t)min(g, pa.K - 1) * F * pa.U];
        for (int k0 = 0; k0 < pa.K; k0 += PG) {
            double2 vn[PG];
#pragma unroll
            for (int g = 0; g < PG; ++g) vn[g] = vq[(size_t)min(k0 + PG + g, pa.K - 1) * F * pa.U];
#pragma unroll
            for (int g = 0; g < PG; ++g) {
                if (k0 + g >= pa.K) break;
                const double* __restrict__ a = aq + (size_t)(k0 + g) * POLY_NA;
#pragma unroll
                for (int j = 0; j <= POLY_IH; ++j) {
                    t[j].x = fma(a[j], vb[g].x, t[j].x);
                    t[j].y = fma(a[j], vb[g].y, t[j].y);
                }
            }
#pragma unroll
            for (int g = 0; g < PG; ++g) vb[g] = vn[g];
        }
        // the taps' loads after the window sums (hoisted above them they would
        // hold 4 IH more registers through the loop)
        __builtin_amdgcn_sched_barrier(0);
        const double2* __restrict__ irq = pa.ir + (size_t)q * pa.N * pa.R + rep;
        if (sh) {
#pragma unroll
            for (int i = 0; i < POLY_IH; ++i) {
                const int n = m + F * (i0 + i);
                if (n < pa.N && i0 + i >= 1) c_fma(r0[i], irq[(size_t)n * pa.R], t[i]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < POLY_IH; ++i) {
                const int n = m + F * (i0 + i);
                if (n < pa.N) c_fma(r0[i], irq[(size_t)n * pa.R], t[i + 1]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // partial fold_k[m] = sum_{i in half} B_k[m + F i] r0[i]
    const double* __restrict__ bm = pa.B + (size_t)m * pa.K * POLY_NI + i0;
    double2* __restrict__ out = (h ? pa.fo2 : pa.fo) + (size_t)m * pa.U + lane;
    for (int k = 0; k < pa.K; ++k) {
        const double* __restrict__ bk = bm + (size_t)k * POLY_NI;
        double2 acc = make_double2(0.0, 0.0);
#pragma unroll
        for (int i = 0; i < POLY_IH; ++i) {
            acc.x = fma(bk[i], r0[i].x, acc.x);
            acc.y = fma(bk[i], r0[i].y, acc.y);
        }
        out[(size_t)k * F * pa.U] = acc;
    }
}

template <int F, class Out>
__global__ void __launch_bounds__(64) k_poly_ana(PolyArgs pa, Out out) {
    extern __shared__ double2 poly_lds[];
    int ug, k;
    poly_block(pa.K, pa.xcd, ug, k);
    const int lane = ug * WAVE + threadIdx.x;
    Out o = out;
    o.prepare(poly_lds);
    double2 x[F];
#pragma unroll
    for (int m = 0; m < F; ++m) {
        const size_t i = (size_t)(k * F + m) * pa.U + lane;
        x[m] = c_add(pa.fo[i], pa.fo2[i]);                    // the two halves' window sums
    }
    const double2* __restrict__ e = pa.E + (size_t)k * F;
    poly_dft<F, -1>(x, pa.tw, [&](int l, double2 y) { o(k * F + l, lane, c_mulf(e[l], y)); });
    o.finish(lane);
}

// eligibility of the polyphase passes (Opts::pic_poly): a factorised scheme,
// F = 24 or 48 (the instantiated DFT sizes), 1-3 taps with delays below F, the
// scratch buffers allocated, whole waves of units
static bool poly_launch_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b) {
    if (!op.pic_poly || !sk.poly_ok || !b.pv || !b.pf || !b.pf2) return false;
    if (sk.poly_F != 24 && sk.poly_F != 48) return false;
    if (sk.poly_F * sk.poly_K != sk.LK || sk.poly_ni > POLY_NI || sk.poly_F * sk.poly_ni < sk.N) return false;
    if (ch.ntap < 1 || ch.ntap > 3) return false;
    for (int q = 0; q < ch.ntap; ++q)
        if (ch.tap_delay[q] < 0 || ch.tap_delay[q] >= sk.poly_F) return false;
    return b.U % WAVE == 0 && b.R % WAVE == 0;
}

static PolyArgs poly_args(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b) {
    PolyArgs pa{};
    pa.u = b.u;
    pa.v = b.pv;
    pa.fo = b.pf;
    pa.fo2 = b.pf2;
    pa.C = sk.poly_C;
    pa.E = sk.poly_E;
    pa.A = sk.poly_A;
    pa.B = sk.poly_B;
    pa.tw = sk.poly_tw;
    pa.ir = b.ir;
    pa.U = b.U;
    pa.R = b.R;
    pa.K = sk.poly_K;
    pa.N = ch.N;
    pa.xcd = op.xcd;
    for (int q = 0; q < 4; ++q) pa.delay[q] = q < ch.ntap ? ch.tap_delay[q] : 0;
    return pa;
}

// t -> r0 -> fold: the first two of the three polyphase launches
static void launch_poly_front(hipStream_t s, const SchemeK& sk, const ChannelK& ch, const PolyArgs& pa) {
    const int ng = pa.U / WAVE;
    const dim3 gs(ng * pa.K), gc(ng * 2 * sk.poly_F), blk(WAVE);
#define POLY_CHAN(FV)                                                                              \
    do {                                                                                           \
        hipLaunchKernelGGL((k_poly_syn<FV>), gs, blk, 0, s, pa);                                   \
        if (ch.ntap == 1) hipLaunchKernelGGL((k_poly_chan<FV, 1>), gc, blk, 0, s, pa);            \
        else if (ch.ntap == 2) hipLaunchKernelGGL((k_poly_chan<FV, 2>), gc, blk, 0, s, pa);       \
        else hipLaunchKernelGGL((k_poly_chan<FV, 3>), gc, blk, 0, s, pa);                         \
    } while (0)
    if (sk.poly_F == 24) POLY_CHAN(24);
    else POLY_CHAN(48);
#undef POLY_CHAN
}

template <class Out>
static void launch_poly_ana(hipStream_t s, const SchemeK& sk, const PolyArgs& pa, const Out& o, size_t lds) {
    const dim3 grid((pa.U / WAVE) * pa.K), blk(WAVE);
    if (sk.poly_F == 24) hipLaunchKernelGGL((k_poly_ana<24, Out>), grid, blk, lds, s, pa, o);
    else hipLaunchKernelGGL((k_poly_ana<48, Out>), grid, blk, lds, s, pa, o);
}

unsigned launch_perfect_ic(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, McBuffers& b,
                           const PerfectDetectArgs* pd) {
    const bool poly = poly_launch_ok(op, sk, ch, b);
    const PolyArgs pa = poly ? poly_args(op, sk, ch, b) : PolyArgs{};
    if (poly) launch_poly_front(s, sk, ch, pa);
    else launch_band(s, sk.G, b.U, nullptr, LoadSoA{b.u, b.U}, StoreSoA{b.t, b.U});
    // SNR-fastest XCD-aware order: the SNR units of a realisation share its taps
    const BandOrder ord{b.U / WAVE, b.U / b.R, b.R / WAVE, op.xcd};
    if (!pd) {
        const StorePerfectIC o{b.yperf, b.y, b.h, b.u, b.U, b.R};
        if (poly) launch_poly_ana(s, sk, pa, o, 0);
        else launch_pass2_nt(s, sk, ch, b, ord, o);
        return poly ? PATH_PIC_POLY : PATH_PIC_PASSES;
    }
    StorePerfectDetect o{};
    o.y = b.y;
    o.h = b.h;
    o.u = b.u;
    o.sidx = b.sidx;
    o.row_data = sk.row_data;
    o.row_cons = sk.row_cons;
    o.row_pval = sk.row_pval;
    o.symbols = sk.symbols;
    o.lvI = sk.lvI;
    o.lvQ = sk.lvQ;
    o.grid_sym = sk.grid_sym;
    o.counters = pd->counters;
    o.cidx0 = ((((size_t)pd->scheme * 2 + 1) * 2 + 0) * pd->nsnr) * pd->nstage + pd->stage;
    o.cstride_edge = pd->nsnr * pd->nstage;
    o.cstride_snr = pd->nstage;
    o.U = b.U;
    o.R = b.R;
    o.rvalid = b.rvalid;
    o.snr0 = b.snr0;
    o.last = pd->last;
    o.M = sk.M;
    o.nI = sk.nI;
    o.nQ = sk.nQ;
    o.real_detect = sk.real_detect;
    o.idd = 1.0 / sk.data_div;
    o.sI = pd->sI;
    o.sQ = pd->sQ;
    o.tr = b.tr;
    o.stage = pd->stage;
    const size_t lds = 256 * sizeof(double2) + sizeof(SlicerLds);
    if (poly) {
        launch_poly_ana(s, sk, pa, o, lds);
        return PATH_PIC_POLY;
    }
    launch_pass2_nt(s, sk, ch, b, ord, o, lds);
    return PATH_PIC_PASSES;
}

// ---------------------------------------------------------------------------
// a13/a15: MMSE contraction  y_est = y - (D_hat - diag h_hat) v  with
// D_hat = sum_p W_p hP_p  (script:417-425, :482-484, :493-511), never forming
// D_hat:  acc[r][u] = sum_{c in band(r)} sum_p W[r, (c,p)] * (hP[p][u] v[c][u]).
// This is a GEMM  [rows x K] * [K x units]  with K = (column, pilot) and the
// right operand Z = hP (x) v generated on the fly; W is shared by all units of
// one SNR point.
//
// VALU variant (one unit per lane, W rows wave-uniform via scalar loads): the
// fallback for pilot counts without a pair-tile instance (NP / 4 not in {2, 4, 8})
// and Opts::wcontract_valu.
__global__ void __launch_bounds__(64) k_wcontract_valu(Band Wb, const double2* __restrict__ Wall, long long w_elems,
                                                       int var, int nsnr, int snr0, int NP, int R, int U,
                                                       const double2* __restrict__ hp, const double2* __restrict__ v,
                                                       const double2* __restrict__ y, double2* __restrict__ yest) {
    extern __shared__ double2 shp[];                     // [NP][64]
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int snr = snr0 + (blockIdx.x * WAVE) / R;
    const int blk = blockIdx.y;
    for (int p = 0; p < NP; ++p) shp[p * WAVE + threadIdx.x] = hp[(size_t)p * U + unit];
    __syncthreads();
    const int row0 = Wb.row0[blk], nrows = Wb.nrows[blk];
    const int c_lo = Wb.klo[blk] / NP, c_hi = Wb.khi[blk] / NP;
    const double2* __restrict__ w = Wall + ((size_t)var * nsnr + snr) * (size_t)w_elems + Wb.off[blk];
    double2 acc[DSCE_WRB];
#pragma unroll
    for (int r = 0; r < DSCE_WRB; ++r) acc[r] = make_double2(0.0, 0.0);
    for (int c = c_lo; c < c_hi; ++c) {
        const double2 vc = v[(size_t)c * U + unit];
        const double2* __restrict__ wc = w + (size_t)(c - c_lo) * NP * DSCE_WRB;
        for (int p = 0; p < NP; ++p) {
            const double2 z = c_mul(shp[p * WAVE + threadIdx.x], vc);
            const double2* __restrict__ wk = wc + (size_t)p * DSCE_WRB;
#pragma unroll
            for (int r = 0; r < DSCE_WRB; ++r) c_fma(acc[r], wk[r], z);
        }
    }
#pragma unroll
    for (int r = 0; r < DSCE_WRB; ++r) {
        if (r < nrows) {
            const size_t i = (size_t)(row0 + r) * U + unit;
            yest[i] = c_sub(y[i], acc[r]);
        }
    }
}

// The W contraction on the matrix cores (k_wpair3), regrouped so no MFMA row is padding.  With
// D_hat[r,c] = sum_p W[(r,c),p] hP_p,  y_est[r] = y[r] - sum_c D_hat[r,c] v_c.
// The first product is a GEMM with M = (row, column) pairs of the block (q = c*RBP
// + r; 24 x 24 pairs of an OFDM symbol tile exactly into 16-pair tiles), K = NP
// and N = units, B = hP constant for the whole block (loaded once); the second
// is applied in the MFMA epilogue: D row (lane>>4)+4*reg of tile t is pair
// 16t + g + 4 reg, whose row index is g (mod 4) for every tile, so each lane
// accumulates RBP/4 rows of its unit with no cross-lane traffic.  Tiles come in
// periods (RBP 24: 3 tiles = 2 columns, RBP 32: 2 tiles = 1 column) so pair ->
// (column, row) is compile-time.  Wave = 16 units, block = 4 waves = 64 units of
// one SNR point; grid (U/64, nblk).
// Complex products in 3M (Gauss / Karatsuba) form: per k-step three real MFMAs
//   P1 += Wr hr,  P2 += Wi hi,  P3 += (Wr + Wi)(hr + hi);  Re = P1 - P2, Im = P3 - P1 - P2
// instead of four (-25 % matrix-core work; the r01 4-MFMA k_wpair was retired in r03); W arrives as three 64-double planes
// per (tile, k-step) (k_wpair_pack3), hP as Re / Im / Re+Im registers.
// Fused MMSE stage (FUSE, block-diagonal W, row-local P): after the
// contraction the tile's rows go straight through the stage of IC iteration
// `stage` instead of being written as y_est and re-read by k_ls + k_stage_fused:
// diag(D_hat) = Wd hP_new on the matrix cores (A = diag(W) rows in MFMA layout,
// B = this stage's LS pilot estimates from k_pilot_pre; its D layout is the
// epilogue's row layout, rows g + 4 k), one-tap y_est ./ h_hat, slicer, error
// counts, and the re-precoded decision written over v (safe in place: with a
// block-diagonal W only this wave reads these rows of v).
struct FuseArgs {
    const double2* WdA;            // [var][snr][blk][2][NKS][64]
    const double2* hp_new;         // this stage's hP [NP][U]
    const uint16_t* sidx;          // transmitted symbol indices [ND][R]
    const double2* h;              // perfect diag(D) [LK][R] (MSE only)
    double2* vout;                 // = v (the re-precoded decisions, in place)
    unsigned long long* counters;
    double* mse_err;
    double* mse_pow;
    const TraceK* tr;              // null unless tracing (dsce_trace_unit_ex)
    int var, stage, nstage, last, scheme;
    int rvalid;                    // realisations of the batch that count (McBuffers::rvalid)
};

template <int RBP, int NKS, bool FUSE>
__device__ __forceinline__ void wpair3_body(const PairBand& P, const double* __restrict__ W3, long long wp_elems,
                                            int var, int nsnr, int snr0, int R, int U,
                                            const double2* __restrict__ hp, const double2* v,
                                            const double2* __restrict__ y, double2* __restrict__ yest,
                                            const SchemeK& sk, const FuseArgs& fa) {
    constexpr int PER = RBP == 24 ? 3 : 2;
    constexpr int CPP = RBP == 24 ? 2 : 1;
    constexpr int NACC = RBP / 4;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int unit = blockIdx.x * 64 + wv * 16 + j;
    const int snr = snr0 + (blockIdx.x * 64) / R;
    const int blk = blockIdx.y;
    __shared__ double2 fsym[FUSE ? 256 : 1];
    __shared__ SlicerLds fslt[1];
    // FUSE: the block's rows (re-precoding value or 0, data index << 1 | no-edge
    // flag or -1) and, per lane, the transmitted symbol indices of its rows
    // (8 bits each, packed) — the epilogue then has no dependent global loads
    __shared__ double2 frpv[FUSE ? RBP : 1];
    __shared__ int frdc[FUSE ? RBP : 1];
    unsigned ftx[FUSE ? 2 : 1] = {0u};
    if (FUSE) {
        stage_tables<256>(fsym, fslt[0], sk, threadIdx.x);
        const int r0b = P.row0[blk], nrb = P.nrows[blk];
        {
            // unconditional loads (clamped row), masked after: see stage_tables
            const int rr = min((int)threadIdx.x, RBP - 1), row = r0b + (rr < nrb ? rr : 0);
            const int dr = sk.row_data[row], pc = sk.row_pcol[row], cs = sk.row_cons[row];
            const double2 pv = sk.row_pval[row];
            const int d = rr < nrb ? dr : -1;
            if (threadIdx.x < RBP) {
                frpv[rr] = make_double2(pc >= 0 ? pv.x : 0.0, pc >= 0 ? pv.y : 0.0);
                frdc[rr] = d >= 0 ? (d << 1) | (cs ? 1 : 0) : -1;
            }
        }
        __syncthreads();
        const int rl0 = (blockIdx.x * 64 + (int)(threadIdx.x >> 6) * 16 + (int)(threadIdx.x & 15)) % R;
        unsigned short tv[NACC];
#pragma unroll
        for (int k = 0; k < NACC; ++k) {
            const int dc = frdc[(threadIdx.x & 63) / 16 + 4 * k < RBP ? (threadIdx.x & 63) / 16 + 4 * k : 0];
            tv[k] = fa.sidx[(size_t)(dc >= 0 ? dc >> 1 : 0) * R + rl0];
        }
#pragma unroll
        for (int k = 0; k < NACC; ++k) ftx[k >> 2] |= ((unsigned)tv[k] & 0xffu) << (8 * (k & 3));
    }
    double br[NKS], bi[NKS], bs[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const double2 h = hp[(size_t)(4 * ks + g) * U + unit];
        br[ks] = h.x;
        bi[ks] = h.y;
        bs[ks] = h.x + h.y;
    }
    const int clo = P.clo[blk], ntile = P.ntile[blk];
    const double* __restrict__ w =
        W3 + ((size_t)var * nsnr + snr) * 3 * (size_t)wp_elems + 3 * P.off[blk] + 2 * lane;
    double2 acc[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = make_double2(0.0, 0.0);
    const double2* __restrict__ vb = v + (size_t)clo * U + unit;
    struct T3 {
        double r[NKS], i[NKS], s[NKS];
    };
    struct D3 {
        d4 p1, p2, p3;
    };
    auto ldt = [&](int t, T3& a) {
        // [tile][k-step pair][plane][lane][2]: one 16-byte load per plane and pair
#pragma unroll
        for (int kp = 0; kp < NKS / 2; ++kp) {
            const double2* q = reinterpret_cast<const double2*>(w + ((size_t)t * (NKS / 2) + kp) * 384);
            const double2 r = q[0], i = q[64], sm = q[128];
            a.r[2 * kp] = r.x;
            a.r[2 * kp + 1] = r.y;
            a.i[2 * kp] = i.x;
            a.i[2 * kp + 1] = i.y;
            a.s[2 * kp] = sm.x;
            a.s[2 * kp + 1] = sm.y;
        }
    };
    auto mma = [&](const T3& a, D3& d) {
        d.p1 = d4{0, 0, 0, 0};
        d.p2 = d.p1;
        d.p3 = d.p1;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            d.p1 = MFMA64(a.r[ks], br[ks], d.p1);
            d.p2 = MFMA64(a.i[ks], bi[ks], d.p2);
            d.p3 = MFMA64(a.s[ks], bs[ks], d.p3);
        }
    };
    // epilogue of a finished tile (period position TT): Re/Im, x v_c, accumulate
    auto epi = [&](const D3& d, const double2 (&vvv)[CPP], auto ttc) {
        constexpr int tt = decltype(ttc)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q0 = 16 * tt + 4 * i;
            const int cc = q0 / RBP, rho = (q0 % RBP) / 4;
            const double re = d.p1[i] - d.p2[i], im = d.p3[i] - d.p1[i] - d.p2[i];
            c_fma(acc[rho], make_double2(re, im), vvv[cc]);
        }
    };
    auto ldv = [&](int per, double2 (&vvv)[CPP]) {
#pragma unroll
        for (int cc = 0; cc < CPP; ++cc) vvv[cc] = vb[(size_t)(per * CPP + cc) * U];
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    // ping-pong W tiles: tile t+1's loads are issued before tile t's MFMAs;
    // sched_barrier keeps the compiler from sinking them back to their uses.
    // RBP 24 runs two periods (6 tiles) per step so the buffers alternate
    // without a register copy (a copy would wait on the just-issued loads).
    T3 A0, A1;
    D3 Da;
    double2 vv[CPP], vw[CPP];
#define WSTEP(LD_T, LD_BUF, MMA_BUF, VV, TT)   \
    ldt(LD_T, LD_BUF);                         \
    __builtin_amdgcn_sched_barrier(0);         \
    mma(MMA_BUF, Da);                          \
    epi(Da, VV, TT{});                         \
    __builtin_amdgcn_sched_barrier(0);
    const int nper = ntile / PER;
    if (ntile > 0) ldt(0, A0);
    if (PER == 3) {
        int per = 0;
        for (; per + 1 < nper; per += 2) {
            const int t0 = per * 3;
            const int tn = t0 + 6 < ntile ? t0 + 6 : t0;
            ldv(per, vv);
            ldv(per + 1, vw);
            WSTEP(t0 + 1, A1, A0, vv, I0)
            WSTEP(t0 + 2, A0, A1, vv, I1)
            WSTEP(t0 + 3, A1, A0, vv, I2)
            WSTEP(t0 + 4, A0, A1, vw, I0)
            WSTEP(t0 + 5, A1, A0, vw, I1)
            WSTEP(tn, A0, A1, vw, I2)
        }
        if (per < nper) {                                   // odd period count: last period
            const int t0 = per * 3;
            ldv(per, vv);
            WSTEP(t0 + 1, A1, A0, vv, I0)
            WSTEP(t0 + 2, A0, A1, vv, I1)
            mma(A0, Da);
            epi(Da, vv, I2{});
        }
    } else {
        for (int t0 = 0; t0 < ntile; t0 += PER) {
            const int tn = t0 + PER < ntile ? t0 + PER : t0;
            ldv(t0 / PER, vv);
            WSTEP(t0 + 1, A1, A0, vv, I0)
            WSTEP(tn, A0, A1, vv, I1)
        }
    }
#undef WSTEP
    const int row0 = P.row0[blk], nrows = P.nrows[blk];
    if (!FUSE) {
#pragma unroll
        for (int k = 0; k < NACC; ++k) {
            const int r = g + 4 * k;
            if (r < nrows) {
                const size_t i = (size_t)(row0 + r) * U + unit;
                yest[i] = c_sub(y[i], acc[k]);
            }
        }
        return;
    }
    // ---- fused stage epilogue -------------------------------------------
    // diag(D_hat) of this stage = Wd hP_new on the matrix cores: B = hP_new in
    // B layout (pilot 4 ks + g, unit j), D rows g + 4 reg + 16 t = this lane's
    // rows g + 4 k of the block.  (Forming it before the tile loop and parking
    // it in LDS measured no faster.)
    d4 er[2], ei[2];
    {
        double hr[NKS], hi[NKS], hs[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const double2 hv = fa.hp_new[(size_t)(4 * ks + g) * U + unit];
            hr[ks] = hv.x;
            hi[ks] = hv.y;
            hs[ks] = hv.x + hv.y;
        }
        const double2* __restrict__ wa = fa.WdA + (((size_t)fa.var * nsnr + snr) * P.nblk + blk) * 2 * NKS * 64 + lane;
        // 3M like the contraction: three real MFMAs per k-step instead of four
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            d4 p1 = d4{0.0, 0.0, 0.0, 0.0}, p2 = p1, p3 = p1;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const double2 a = wa[(t * NKS + ks) * 64];
                p1 = MFMA64(a.x, hr[ks], p1);
                p2 = MFMA64(a.y, hi[ks], p2);
                p3 = MFMA64(a.x + a.y, hs[ks], p3);
            }
            er[t] = p1 - p2;
            ei[t] = p3 - p1 - p2;
        }
    }
    const int rl = unit % R;
    const double idd = 1.0 / sk.data_div;
    int cnt[4] = {0, 0, 0, 0};
    double me = 0.0, mp = 0.0;
    // all rows' y requested first and every row computed, padding / pilot rows
    // masked afterwards (a per-row branch lets the compiler sink each y load
    // into it: one serial round trip per row)
    double2 yv[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
        const int r = g + 4 * k;
        yv[k] = y[(size_t)(row0 + (r < nrows ? r : 0)) * U + unit];
    }
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
        const int r = g + 4 * k;
        const bool valid = r < nrows;
        const int row = row0 + (valid ? r : 0);
        const size_t ix = (size_t)row * U + unit;
        const double2 ye = c_sub(yv[k], acc[k]);
        const double2 he = make_double2(er[k >> 2][k & 3], ei[k >> 2][k & 3]);
        if (fa.mse_err && valid) {
            const double2 hv = fa.h[(size_t)row * R + rl];
            const double dx = he.x - hv.x, dy = he.y - hv.y;
            me += dx * dx + dy * dy;
        }
        const int dc = valid ? frdc[r] : -1;
        const double2 z = c_div1(ye, he);
        const int de = slice_fast(fslt[0], sk.nI, sk.nQ,
                                  sk.real_detect ? make_double2(z.x * idd, 0.0) : make_double2(z.x * idd, z.y * idd),
                                  sk.slI, sk.slQ);
        const int ne = dc >= 0 ? __popc((unsigned)(de ^ (int)((ftx[k >> 2] >> (8 * (k & 3))) & 0xffu))) : 0;
        cnt[0] += ne;
        cnt[1] += (dc & 1) ? ne : 0;
        if (fa.tr && valid && unit == fa.tr->unit) {
            fa.tr->yest[(size_t)fa.stage * fa.tr->LK + row] = ye;
            fa.tr->hest[(size_t)fa.stage * fa.tr->LK + row] = he;
            if (dc >= 0) fa.tr->dec_e[(size_t)fa.stage * fa.tr->ND + (dc >> 1)] = de;
        }
        if (!fa.last && dc >= 0) {
            double2 av = make_double2(0.0, 0.0);
            c_fma(av, frpv[valid ? r : 0], fsym[de]);
            fa.vout[ix] = av;
        }
    }
    flush_counts(cnt, fa.counters, (((size_t)fa.scheme * 4) * nsnr + snr) * fa.nstage + fa.stage,
                 (size_t)nsnr * fa.nstage, 1, rl < fa.rvalid);
    if (fa.mse_err) flush_mse(me, mp, fa.mse_err, fa.mse_pow, fa.scheme, nsnr, snr, fa.nstage, fa.stage, rl < fa.rvalid);
}

template <int RBP, int NKS, bool FUSE>
__global__ void __launch_bounds__(256)
    k_wpair3(PairBand P, const double* __restrict__ W3, long long wp_elems, int var, int nsnr, int snr0, int R, int U,
             const double2* __restrict__ hp, const double2* v, const double2* __restrict__ y,
             double2* __restrict__ yest, SchemeK sk, FuseArgs fa) {
    wpair3_body<RBP, NKS, FUSE>(P, W3, wp_elems, var, nsnr, snr0, R, U, hp, v, y, yest, sk, fa);
}

// The unfused W contraction of 32-row blocks (FBMC, C5) as ONE GEMM per row
// tile (k_wrow3, Opts::wrow): y_est[r] = y[r] - sum_(c,p) W[(r,c),p] X[(c,p)]
// with X[(c,p)] = hP_p v_c per unit.  M = the block's rows (two 16-row tiles),
// K = (column, pilot), N = units: the pair tile t = 2 c + h of k_wpair3's
// storage IS the A fragment of row tile h and column c (pairs q = 32 c + r), so
// the same W3 planes feed it.  The accumulators (3M: P1, P2, P3 per row tile)
// stay in registers over every column of the band and the complex
// D_hat[r,c] v_c epilogue of each tile disappears: per column the VALU forms
// X = hP v_c once (NKS complex products, shared by both row tiles) instead of
// 2 x 4 complex MACs plus the 3M recombination per tile (k_wpair3: 17 % of the
// issue next to 3 NKS MFMAs per tile at C3 / C4).  Same flops, other rounding
// order (parity to 1e-9 like every contraction path).
template <int NKS>
__global__ void __launch_bounds__(256)
    k_wrow3(PairBand P, const double* __restrict__ W3, long long wp_elems, int var, int nsnr, int snr0, int R, int U,
            const double2* __restrict__ hp, const double2* __restrict__ v, const double2* __restrict__ y,
            double2* __restrict__ yest) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int unit = blockIdx.x * 64 + wv * 16 + j;
    const int snr = snr0 + (blockIdx.x * 64) / R;
    const int blk = blockIdx.y;
    double2 hpl[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) hpl[ks] = hp[(size_t)(4 * ks + g) * U + unit];
    const int clo = P.clo[blk], ntile = P.ntile[blk];
    const double* __restrict__ w =
        W3 + ((size_t)var * nsnr + snr) * 3 * (size_t)wp_elems + 3 * P.off[blk] + 2 * lane;
    const double2* __restrict__ vb = v + (size_t)clo * U + unit;
    struct T3 {
        double r[NKS], i[NKS], s[NKS];
    };
    auto ldt = [&](int t, T3& a) {
#pragma unroll
        for (int kp = 0; kp < NKS / 2; ++kp) {
            const double2* q = reinterpret_cast<const double2*>(w + ((size_t)t * (NKS / 2) + kp) * 384);
            const double2 r = q[0], i = q[64], sm = q[128];
            a.r[2 * kp] = r.x;
            a.r[2 * kp + 1] = r.y;
            a.i[2 * kp] = i.x;
            a.i[2 * kp + 1] = i.y;
            a.s[2 * kp] = sm.x;
            a.s[2 * kp + 1] = sm.y;
        }
    };
    double xr[NKS], xi[NKS], xs[NKS];
    auto formx = [&](double2 vc) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const double2 xv = c_mulf(hpl[ks], vc);
            xr[ks] = xv.x;
            xi[ks] = xv.y;
            xs[ks] = xv.x + xv.y;
        }
    };
    d4 p[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 3; ++k) p[h][k] = d4{0.0, 0.0, 0.0, 0.0};
    auto mma = [&](const T3& a, auto hc) {
        constexpr int h = decltype(hc)::value;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            p[h][0] = MFMA64(a.r[ks], xr[ks], p[h][0]);
            p[h][1] = MFMA64(a.i[ks], xi[ks], p[h][1]);
            p[h][2] = MFMA64(a.s[ks], xs[ks], p[h][2]);
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // ping-pong W tiles (tile t + 1's loads issued before tile t's MFMAs) and v
    // one column ahead; a column is two tiles (row tiles 0 and 1)
    T3 A0, A1;
    const int ncol = ntile / 2;
    double2 vn = ncol > 0 ? vb[0] : make_double2(0.0, 0.0);
    if (ntile > 0) ldt(0, A0);
    for (int c = 0; c < ncol; ++c) {
        const int t0 = 2 * c;
        formx(vn);
        vn = vb[(size_t)(c + 1 < ncol ? c + 1 : c) * U];
        ldt(t0 + 1, A1);
        __builtin_amdgcn_sched_barrier(0);
        mma(A0, I0{});
        __builtin_amdgcn_sched_barrier(0);
        ldt(t0 + 2 < ntile ? t0 + 2 : t0 + 1, A0);
        __builtin_amdgcn_sched_barrier(0);
        mma(A1, I1{});
        __builtin_amdgcn_sched_barrier(0);
    }
    const int row0 = P.row0[blk], nrows = P.nrows[blk];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 16 * h + g + 4 * i;
            if (r < nrows) {
                const size_t ix = (size_t)(row0 + r) * U + unit;
                const double re = p[h][0][i] - p[h][1][i], im = p[h][2][i] - p[h][0][i] - p[h][1][i];
                yest[ix] = c_sub(y[ix], make_double2(re, im));
            }
        }
}

// Pre-pass of the fused MMSE stage of IC iteration `stage` (script:482-489):
// y_est at the NP pilot rows with the previous stage's D_hat (W of var_prev,
// the contraction's), then the LS estimates hP = y_est(pilots) ./ xP /
// sqrt(kappa) into hp_new, which the fused contraction's epilogue needs
// before any row can be detected.  Lane = unit; the pilot rows of W stream
// with wave-uniform (scalar) loads.  NP x 24 x (NP + 1) CMACs per unit, 5 % of
// the contraction.
template <int NP>
__global__ void __launch_bounds__(64) k_pilot_pre(SchemeK sk, const double2* __restrict__ Wpil,
                                                  const int* __restrict__ pil_c0, int var_prev, int nsnr, int snr0,
                                                  int R, int U, const double2* __restrict__ hp_prev,
                                                  const double2* __restrict__ v, const double2* __restrict__ y,
                                                  const double2* __restrict__ xp, double2* __restrict__ hp_new) {
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int rl = unit % R;
    const int snr = snr0 + (blockIdx.x * WAVE) / R;
    // column c of v = P [xP; Q(x_est)] (c is wave-uniform: the row tables are
    // scalar loads)
    auto vcol = [&](int c) -> double2 { return v[(size_t)c * U + unit]; };
    double2 hq[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) hq[p] = hp_prev[(size_t)p * U + unit];
    const double2* __restrict__ wb = Wpil + ((size_t)var_prev * nsnr + snr) * (size_t)NP * 24 * NP;
    const double sqk = 1.0 / sk.inv_sqrt_kappa;
    for (int i = 0; i < NP; ++i) {
        const int r = sk.pilot_pos[i], c0 = pil_c0[i];
        const double2* __restrict__ wi = wb + (size_t)i * 24 * NP;
        // D_hat[r, c] = sum_p W hP_p in 4 partial sums (independent FMA chains),
        // two columns per step
        double2 acc = make_double2(0.0, 0.0);
        for (int cc = 0; cc < 24; cc += 2) {
            const double2 va = vcol(c0 + cc);
            const double2 vb = vcol(c0 + cc + 1);
            double2 d[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) d[k] = make_double2(0.0, 0.0);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                c_fma(d[p & 3], wi[cc * NP + p], hq[p]);
                c_fma(d[4 + (p & 3)], wi[(cc + 1) * NP + p], hq[p]);
            }
            c_fma(acc, c_add(c_add(d[0], d[1]), c_add(d[2], d[3])), va);
            c_fma(acc, c_add(c_add(d[4], d[5]), c_add(d[6], d[7])), vb);
        }
        const double2 ye = c_sub(y[(size_t)r * U + unit], acc);
        const double2 q = c_div(ye, xp[(size_t)i * R + rl]);
        hp_new[(size_t)i * U + unit] = make_double2(q.x / sqk, q.y / sqk);
    }
}

bool mmse_fused_ok(const Opts& op, const SchemeK& sk, const MmseK& mm, const McBuffers& b) {
    return mm.Wpil && mm.WdA && mm.Pb.rbp == 24 && mm.Pb.nks == 4 && sk.NP == 16 && op.fuse_stage &&
           !op.wcontract_valu && mm.Wp3 && (b.U % 64) == 0 && (b.R % 64) == 0;
}

void launch_pilot_pre(hipStream_t s, const SchemeK& sk, const MmseK& mm, int var_prev, McBuffers& b,
                      const double2* hp_prev, double2* hp_new) {
    hipLaunchKernelGGL((k_pilot_pre<16>), dim3(b.U / WAVE), dim3(WAVE), 0, s, sk, mm.Wpil, mm.pil_c0, var_prev, mm.nsnr,
                       b.snr0, b.R, b.U, hp_prev, b.v, b.y, b.xp, hp_new);
}

unsigned launch_mmse_fused(hipStream_t s, const Opts& op, const SchemeK& sk, const MmseK& mm, int var_prev,
                           int var_cur, int stage, int n_iter, bool last, McBuffers& b, const double2* hp_prev,
                           double2* hp_new, unsigned long long* counters, int scheme_index) {
    FuseArgs fa{};
    fa.WdA = mm.WdA;
    fa.hp_new = hp_new;
    fa.sidx = b.sidx;
    fa.h = b.h;
    fa.vout = b.v;
    fa.counters = counters;
    fa.mse_err = b.mse_err;
    fa.mse_pow = b.mse_pow;
    fa.tr = b.tr;
    fa.var = var_cur;
    fa.stage = stage;
    fa.nstage = n_iter + 1;
    fa.last = last ? 1 : 0;
    fa.scheme = scheme_index;
    fa.rvalid = b.rvalid;
    const dim3 grid(b.U / 64, mm.Pb.nblk);
    hipLaunchKernelGGL((k_wpair3<24, 4, true>), grid, dim3(256), 0, s, mm.Pb, mm.Wp3, mm.wp_elems, var_prev, mm.nsnr,
                       b.snr0, b.R, b.U, hp_prev, b.v, b.y, b.yest, sk, fa);
    return PATH_WPAIR3_FUSED;
}

unsigned launch_wcontract(hipStream_t s, const Opts& op, const SchemeK& sk, const MmseK& mm, int var, McBuffers& b) {
    // the pair-tile contraction (k_wpair3), or the VALU contraction over the
    // packed band where no pair tiles exist (a block wider than 32 rows) or on
    // request (Opts::wcontract_valu)
    const bool pair_ok = mm.Wp3 && (b.U % 64) == 0 && (b.R % 64) == 0 && !op.wcontract_valu;
    if (pair_ok && op.wrow && mm.Pb.rbp == 32) {
        // 32-row blocks: one GEMM per row tile, no per-tile epilogue (k_wrow3)
        const dim3 grid(b.U / 64, mm.Pb.nblk);
#define LAUNCH_WR(NKSV)                                                                                            \
    hipLaunchKernelGGL((k_wrow3<NKSV>), grid, dim3(256), 0, s, mm.Pb, mm.Wp3, mm.wp_elems, var, mm.nsnr, b.snr0, b.R, \
                       b.U, b.hp, b.v, b.y, b.yest)
        if (mm.Pb.nks == 2) LAUNCH_WR(2);
        else if (mm.Pb.nks == 4) LAUNCH_WR(4);
        else LAUNCH_WR(8);
#undef LAUNCH_WR
        return PATH_WROW3;
    }
    if (pair_ok) {
        const dim3 grid(b.U / 64, mm.Pb.nblk);
#define LAUNCH_W3(RBPV, NKSV)                                                                                  \
    hipLaunchKernelGGL((k_wpair3<RBPV, NKSV, false>), grid, dim3(256), 0, s, mm.Pb, mm.Wp3, mm.wp_elems, var,    \
                       mm.nsnr, b.snr0, b.R, b.U, b.hp, b.v, b.y, b.yest, sk, FuseArgs{})
        if (mm.Pb.rbp == 24) {
            if (mm.Pb.nks == 2) LAUNCH_W3(24, 2);
            else if (mm.Pb.nks == 4) LAUNCH_W3(24, 4);
            else LAUNCH_W3(24, 8);
        } else {
            if (mm.Pb.nks == 2) LAUNCH_W3(32, 2);
            else if (mm.Pb.nks == 4) LAUNCH_W3(32, 4);
            else LAUNCH_W3(32, 8);
        }
#undef LAUNCH_W3
        return PATH_WPAIR3;
    }
    hipLaunchKernelGGL(k_wcontract_valu, dim3(b.U / WAVE, mm.Wb.nblk), dim3(WAVE), sk.NP * WAVE * sizeof(double2), s,
                       mm.Wb, mm.W, mm.w_elems, var, mm.nsnr, b.snr0, sk.NP, b.R, b.U, b.hp, b.v, b.y, b.yest);
    return PATH_WCONTRACT_VALU;
}

// ---------------------------------------------------------------------------
// a14/a16: one stage of the receiver (one-tap or IC iteration), lane = unit:
// LS at the pilots (script:412-414 / :487-489), h_hat = diag(D_hat)
// (script:428 / :515), one-tap equalisation + detection (SignalConstellation.m:83-101,
// first minimum wins), error counting with and without edges (script:432-447 /
// :531-537 / :548-561), and re-precoding of the quantised decisions for the next
// IC iteration (script:482-484 / :541-543).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int nearest_level(const double* __restrict__ lv, int n, double x, int& alt) {
    alt = -1;
    if (n == 1) return 0;
    const double step = lv[1] - lv[0];
    int i = (int)floor((x - lv[0]) / step);
    i = i < 0 ? 0 : (i > n - 2 ? n - 2 : i);
    const double d0 = fabs(x - lv[i]), d1 = fabs(x - lv[i + 1]);
    if (d1 < d0) return i + 1;
    if (d1 == d0) alt = i + 1;
    return i;
}

__device__ __forceinline__ int slice(const SchemeK& sk, double2 z) {
    int aI, aQ;
    const int iI = nearest_level(sk.lvI, sk.nI, z.x, aI);
    const int iQ = nearest_level(sk.lvQ, sk.nQ, z.y, aQ);
    int best = sk.grid_sym[iI * sk.nQ + iQ];
    if (aI >= 0) best = min(best, sk.grid_sym[aI * sk.nQ + iQ]);
    if (aQ >= 0) best = min(best, sk.grid_sym[iI * sk.nQ + aQ]);
    if (aI >= 0 && aQ >= 0) best = min(best, sk.grid_sym[aI * sk.nQ + aQ]);
    return best;
}

struct StageArgs {
    int stage, var, nsnr, nstage, scheme, last, perfect, R, U, snr0, xcd_order;
    int rvalid;                // realisations of the batch that count (McBuffers::rvalid)
    const TraceK* tr;          // null unless tracing (dsce_trace_unit_ex)
    const double2* ysrc_e;     // y (stage 0) or y_est
    const double2* ysrc_p;     // y (stage 0) or y_perf
    double* mse_err;           // null: no MSE accumulation (see flush_mse)
    double* mse_pow;
};

// (1) h_hat = diag(D_hat) = sum_p W[(c,c),p] hP_p and the one-tap quotients
// y./h_hat (MMSE) and y./h (perfect CSI) for a block of DSCE_RB rows, from the
// LS pilot estimates k_ls wrote (r04: each row block recomputed the NP complex
// LS divisions itself, and wrote h_hat, which nothing reads, to HBM);
// grid (U/64, ceil(LK/RB)).
__global__ void __launch_bounds__(64) k_ls_hest(SchemeK sk, StageArgs st, const double2* __restrict__ Wd,
                                                const double2* __restrict__ h, const double2* __restrict__ hp,
                                                double2* __restrict__ e_est, double2* __restrict__ e_perf) {
    extern __shared__ double2 shp[];                     // [NP][64], each lane its own column
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int snr = st.snr0 + (blockIdx.x * WAVE) / st.R;
    const int rl = unit % st.R;
    const int U = st.U, R = st.R;
    for (int p = 0; p < sk.NP; ++p) shp[p * WAVE + threadIdx.x] = hp[(size_t)p * U + unit];
    const double2* __restrict__ wd = Wd + ((size_t)st.var * st.nsnr + snr) * (size_t)sk.LK * sk.NP;
    const int r0 = blockIdx.y * DSCE_RB;
    const int r1 = min(sk.LK, r0 + DSCE_RB);
    double me = 0.0, mp = 0.0;
    for (int c = r0; c < r1; ++c) {
        double2 acc = make_double2(0.0, 0.0);
        for (int p = 0; p < sk.NP; ++p) c_fma(acc, wd[(size_t)c * sk.NP + p], shp[p * WAVE + threadIdx.x]);
        const size_t i = (size_t)c * U + unit;
        const double2 hv = h[(size_t)c * R + rl];
        if (st.tr && unit == st.tr->unit) st.tr->hest[(size_t)st.stage * st.tr->LK + c] = acc;
        e_est[i] = c_div(st.ysrc_e[i], acc);
        e_perf[i] = c_div(st.ysrc_p[i], hv);
        if (st.mse_err) {
            const double dx = acc.x - hv.x, dy = acc.y - hv.y;
            me += dx * dx + dy * dy;
            mp += hv.x * hv.x + hv.y * hv.y;
        }
    }
    if (st.mse_err) flush_mse(me, mp, st.mse_err, st.mse_pow, st.scheme, st.nsnr, snr, st.nstage, st.stage, rl < st.rvalid);
}

// (2) data-symbol decisions and bit-error counts, grid (U/64, ceil(ND/32)).
static constexpr int DET_CHUNK = 32;
__global__ void __launch_bounds__(64) k_detect(SchemeK sk, StageArgs st, const uint16_t* __restrict__ sidx,
                                               const double2* __restrict__ e_est, const double2* __restrict__ e_perf,
                                               uint16_t* __restrict__ qe, uint16_t* __restrict__ qp,
                                               unsigned long long* __restrict__ counters) {
    __shared__ SlicerLds slt;
    const bool lds_slicer = sk.nI <= 16 && sk.nQ <= 16;
    if (lds_slicer) slicer_load(slt, sk, threadIdx.x, WAVE);
    __syncthreads();
    const double sI = sk.slI, sQ = sk.slQ;
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int snr = st.snr0 + (blockIdx.x * WAVE) / st.R;
    const int rl = unit % st.R;
    const int U = st.U, R = st.R;
    const int i0 = blockIdx.y * DET_CHUNK;
    const int i1 = min(sk.ND, i0 + DET_CHUNK);
    int cnt[4] = {0, 0, 0, 0};
    for (int csi = 0; csi < 2; ++csi) {
        const double2* __restrict__ e = csi == 0 ? e_est : e_perf;
        uint16_t* __restrict__ qo = csi == 0 ? qe : qp;
        for (int i = i0; i < i1; ++i) {
            double2 z;
            if (sk.despread) {                                  // x = P' (y ./ h), script:436 / :520
                const int row = sk.NP + i;
                double2 acc = make_double2(0.0, 0.0);
                // entries in groups of 4, every load of a group issued before its
                // products (one global round trip per group instead of per entry)
                const int j0 = sk.ph_ptr[row], j1 = sk.ph_ptr[row + 1];
                for (int jb = j0; jb < j1; jb += 4) {
                    double2 ev[4], pv[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int jj = min(jb + g, j1 - 1);
                        pv[g] = jb + g < j1 ? sk.ph_val[jj] : make_double2(0.0, 0.0);
                        ev[g] = e[(size_t)sk.ph_col[jj] * U + unit];
                    }
#pragma unroll
                    for (int g = 0; g < 4; ++g) c_fma(acc, pv[g], ev[g]);
                }
                z = acc;
                z = sk.real_detect ? make_double2(z.x / sk.data_div, 0.0)
                                   : make_double2(z.x / sk.data_div, z.y / sk.data_div);
            } else {                                            // x(data positions) ./ sqrt(DPR)
                z = e[(size_t)sk.data_pos[i] * U + unit];
                z = sk.real_detect ? make_double2(z.x / sk.data_div, 0.0)
                                   : make_double2(z.x / sk.data_div, z.y / sk.data_div);
            }
            const int d = lds_slicer ? slice_fast(slt, sk.nI, sk.nQ, z, sI, sQ) : slice(sk, z);
            const int tx = sidx[(size_t)i * R + rl];
            const int ne = __popc((unsigned)(d ^ tx));
            if (st.tr && unit == st.tr->unit) (csi ? st.tr->dec_p : st.tr->dec_e)[(size_t)st.stage * st.tr->ND + i] = d;
            cnt[csi * 2 + 0] += ne;
            if (sk.considered[i]) cnt[csi * 2 + 1] += ne;
            if (!st.last) qo[(size_t)i * U + unit] = (uint16_t)d;
        }
    }
    flush_counts(cnt, counters, (((size_t)st.scheme * 4) * st.nsnr + snr) * st.nstage + st.stage,
                 (size_t)st.nsnr * st.nstage, 2, rl < st.rvalid);
}

// (3) re-precoding of the quantised decisions for the next IC iteration:
// v = P [xP; Q(x_est)], u = P [xP; Q(x_perf)] (script:482-484, :541-543);
// grid (U/64, ceil(LK/24)).
__global__ void __launch_bounds__(64) k_precode(SchemeK sk, StageArgs st, const double2* __restrict__ xp,
                                                const uint16_t* __restrict__ qe, const uint16_t* __restrict__ qp,
                                                double2* __restrict__ v, double2* __restrict__ u) {
    __shared__ double2 sym[256];
    for (int i = threadIdx.x; i < sk.M; i += WAVE) sym[i] = sk.symbols[i];
    __syncthreads();
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int rl = unit % st.R;
    const int U = st.U, R = st.R;
    const int r0 = blockIdx.y * DSCE_RB;
    const int r1 = min(sk.LK, r0 + DSCE_RB);
    for (int r = r0; r < r1; ++r) {
        double2 av = make_double2(0.0, 0.0), au = make_double2(0.0, 0.0);
        const int j0 = sk.p_ptr[r], j1 = sk.p_ptr[r + 1];
        // entries in groups of PJ: every index / pilot load of a group is issued
        // before the first LDS lookup (a row of the auxiliary-symbol precoder has
        // ~30 entries; one dependent global -> LDS -> FMA round trip per entry
        // left the kernel latency-bound, r04: 4.3 ms per C3 launch)
        constexpr int PJ = 4;
        for (int jb = j0; jb < j1; jb += PJ) {
            int ie[PJ], iq[PJ];
            double2 xv[PJ];
#pragma unroll
            for (int g = 0; g < PJ; ++g) {
                const int k = sk.p_col[min(jb + g, j1 - 1)];
                if (k < sk.NP) {                                  // uniform branch
                    xv[g] = xp[(size_t)k * R + rl];
                    ie[g] = iq[g] = -1;
                } else {
                    xv[g] = make_double2(0.0, 0.0);
                    ie[g] = qe[(size_t)(k - sk.NP) * U + unit];
                    iq[g] = qp[(size_t)(k - sk.NP) * U + unit];
                }
            }
#pragma unroll
            for (int g = 0; g < PJ; ++g) {
                if (jb + g >= j1) break;                          // uniform
                const double2 pv = sk.p_val[jb + g];
                c_fma(av, pv, ie[g] >= 0 ? sym[ie[g]] : xv[g]);
                c_fma(au, pv, iq[g] >= 0 ? sym[iq[g]] : xv[g]);
            }
        }
        v[(size_t)r * U + unit] = av;
        u[(size_t)r * U + unit] = au;
    }
}

// LS pilot estimates alone (script:412-414 / :487-489), lane = unit; grid U/64.
__global__ void __launch_bounds__(64) k_ls(SchemeK sk, StageArgs st, const double2* __restrict__ xp,
                                           double2* __restrict__ hp) {
    const int unit = blockIdx.x * WAVE + threadIdx.x;
    const int rl = unit % st.R;
    const double sqk = 1.0 / sk.inv_sqrt_kappa;
    for (int p = 0; p < sk.NP; ++p) {
        const double2 q = c_div(st.ysrc_e[(size_t)sk.pilot_pos[p] * st.U + unit], xp[(size_t)p * st.R + rl]);
        hp[(size_t)p * st.U + unit] = make_double2(q.x / sqk, q.y / sqk);
    }
}

// Fused stage for select-mode schemes (OFDM, FBMC auxiliary), one pass over a
// block of RB rows: diag(D_hat) = Wd hP (p-outer, RB accumulators, Wd rows
// wave-uniform), one-tap quotients, slicing + error counts for both CSI
// branches, and either the row-local re-precoding v / u (p_diag, OFDM) or the
// decisions for k_precode.  diag(D_hat) is written only for traces; the
// contraction uses a W band with a zero diagonal, so nothing else reads it.
// Flat grid, row block fastest (the blocks of one unit group share hP in L2).
template <int NPT, int RB, bool PERF, bool MSE>
__global__ void __launch_bounds__(256) k_stage_fused(SchemeK sk, StageArgs st, int nrb, const double2* __restrict__ Wd,
                                                     const double2* __restrict__ xp,
                                                     const uint16_t* __restrict__ sidx,
                                                     const double2* __restrict__ h,
                                                     const double2* __restrict__ hp, double2* __restrict__ hest,
                                                     uint16_t* __restrict__ qe, uint16_t* __restrict__ qp,
                                                     double2* __restrict__ v, double2* __restrict__ u,
                                                     unsigned long long* __restrict__ counters) {
    __shared__ double2 sym[256];
    __shared__ SlicerLds slt;
    __shared__ double2 shp[NPT * 64];                      // the block's 64 units' LS pilot estimates
    __shared__ double2 swd[4 * RB * NPT];                  // diag(W) rows of the block (broadcast reads)
    // Block = 64 units x 4*RB rows (wave w: rows [4 RB blk + w RB, +RB)); the LS
    // pilot estimates of the 64 units go through LDS once for the 4 waves.
    // Work order: row block fastest, then SNR point, then 64-realisation group,
    // so the blocks sharing hP (same units) and h (same realisations) run close
    // together; with xcd_order each XCD (block b runs on XCD b % 8) walks its own
    // contiguous range of that order, keeping the reuse inside one L2.
    int L = blockIdx.x;
    if (st.xcd_order) L = xcd_remap(L, gridDim.x);
    const int rbk = L % nrb;
    int ug = L / nrb;
    if (st.xcd_order) {
        const int nchunk = st.U / st.R, rgs = st.R >> 6;
        ug = (ug % nchunk) * rgs + ug / nchunk;
    }
    // wave index made provably uniform so Wd / row tables become scalar loads
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int U = st.U, R = st.R;
    const int unit = ug * 64 + lane;
    const int snr = st.snr0 + (ug * 64) / R;
    const int rl = unit % R;
    const int r0 = (rbk * 4 + wv) * RB;
    const int nr = max(0, min(RB, sk.LK - r0));
    // every per-row operand of the wave is requested up front (rows past the
    // end / pilot rows read a valid dummy), so their latency overlaps diag(D_hat)
    double2 ye[RB], yp[RB], hh[RB];
    int tx[RB];
    const bool same_y = st.ysrc_p == st.ysrc_e;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int row = r < nr ? r0 + r : 0;
        const int i = sk.row_data[row];
        const size_t ix = (size_t)row * U + unit;
        ye[r] = st.ysrc_e[ix];
        tx[r] = sidx[(size_t)(i > 0 ? i : 0) * R + rl];
        if (PERF) yp[r] = same_y ? ye[r] : st.ysrc_p[ix];
        if (PERF || MSE) hh[r] = h[(size_t)row * R + rl];
    }
    // per-row scalars of the wave's rows, requested together (no dependent chains)
    int rdat[RB], rcons[RB], rpcol[RB];
    double2 rpval[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int row = r < nr ? r0 + r : 0;
        rdat[r] = sk.row_data[row];
        rcons[r] = sk.row_cons[row];
        rpcol[r] = sk.row_pcol[row];
        rpval[r] = sk.row_pval[row];
    }
    {
        // LDS staging: hP of the 64 units, diag(W) rows of the block, tables;
        // every global load is issued before the first LDS write
        constexpr int NW = (4 * RB * NPT + 255) / 256;
        double2 hv[NPT / 4], wv_[NW];
#pragma unroll
        for (int k = 0; k < NPT / 4; ++k) {
            const int i = threadIdx.x + 256 * k;
            hv[k] = hp[(size_t)(i >> 6) * U + ug * 64 + (i & 63)];
        }
        const int rb0 = rbk * 4 * RB;
        const double2* __restrict__ wdb = Wd + ((size_t)st.var * st.nsnr + snr) * (size_t)sk.LK * NPT;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int i = threadIdx.x + 256 * k;
            const int row = rb0 + i / NPT;
            wv_[k] = (i < 4 * RB * NPT && row < sk.LK) ? wdb[(size_t)rb0 * NPT + i] : make_double2(0.0, 0.0);
        }
        stage_tables<256>(sym, slt, sk, threadIdx.x);
#pragma unroll
        for (int k = 0; k < NPT / 4; ++k) shp[threadIdx.x + 256 * k] = hv[k];
#pragma unroll
        for (int k = 0; k < NW; ++k)
            if (threadIdx.x + 256 * k < 4 * RB * NPT) swd[threadIdx.x + 256 * k] = wv_[k];
    }
    __syncthreads();
    if (nr == 0) return;
    const double2* __restrict__ wds = swd + wv * RB * NPT;
    double2 acc[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = make_double2(0.0, 0.0);
#pragma unroll
    for (int p = 0; p < NPT; ++p) {
        const double2 hv = shp[p * 64 + lane];
#pragma unroll
        for (int r = 0; r < RB; ++r)
            if (r < nr) c_fma(acc[r], wds[r * NPT + p], hv);
    }
    if (MSE) {
        double me = 0.0, mp = 0.0;
#pragma unroll
        for (int r = 0; r < RB; ++r)
            if (r < nr) {
                const double dx = acc[r].x - hh[r].x, dy = acc[r].y - hh[r].y;
                me += dx * dx + dy * dy;
                mp += hh[r].x * hh[r].x + hh[r].y * hh[r].y;
            }
        flush_mse(me, mp, st.mse_err, st.mse_pow, st.scheme, st.nsnr, snr, st.nstage, st.stage, rl < st.rvalid);
    }
    const double idd = 1.0 / sk.data_div;
    const double sI = sk.slI, sQ = sk.slQ;
    int cnt[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        if (r < nr) {
            const int row = r0 + r;
            const size_t ix = (size_t)row * U + unit;
            const bool traced = st.tr && unit == st.tr->unit;
            if (traced) st.tr->hest[(size_t)st.stage * st.tr->LK + row] = acc[r];
            const int i = rdat[r];
            if (i >= 0) {
                const double2 ze = c_div1(ye[r], acc[r]);
                const int de = slice_fast(slt, sk.nI, sk.nQ, sk.real_detect ? make_double2(ze.x * idd, 0.0)
                                                             : make_double2(ze.x * idd, ze.y * idd), sI, sQ);
                const int ne = __popc((unsigned)(de ^ tx[r]));
                const int cons = rcons[r];
                cnt[0] += ne;
                cnt[1] += cons ? ne : 0;
                int dp = 0;
                if (PERF) {
                    const double2 zp = c_div1(yp[r], hh[r]);
                    dp = slice_fast(slt, sk.nI, sk.nQ, sk.real_detect ? make_double2(zp.x * idd, 0.0)
                                                      : make_double2(zp.x * idd, zp.y * idd), sI, sQ);
                    const int np_ = __popc((unsigned)(dp ^ tx[r]));
                    cnt[2] += np_;
                    cnt[3] += cons ? np_ : 0;
                }
                if (traced) {
                    st.tr->dec_e[(size_t)st.stage * st.tr->ND + i] = de;
                    if (PERF) st.tr->dec_p[(size_t)st.stage * st.tr->ND + i] = dp;
                }
                if (!st.last) {
                    if (sk.p_diag) {
                        const double2 pv = rpval[r];
                        double2 av = make_double2(0.0, 0.0), au = av;
                        if (rpcol[r] >= 0) {
                            c_fma(av, pv, sym[de]);
                            c_fma(au, pv, sym[dp]);
                        }
                        v[ix] = av;
                        if (PERF) u[ix] = au;
                    } else {
                        const size_t qi = (size_t)i * U + unit;
                        qe[qi] = (uint16_t)de;
                        qp[qi] = (uint16_t)dp;
                    }
                }
            } else if (!st.last && sk.p_diag && st.stage == 0) {   // pilot / empty row: constant P xP
                const int kc = rpcol[r];
                double2 av = make_double2(0.0, 0.0);
                if (kc >= 0) c_fma(av, rpval[r], xp[(size_t)kc * R + rl]);
                v[ix] = av;
                u[ix] = av;
            }
        }
    }
    flush_counts(cnt, counters, (((size_t)st.scheme * 4) * st.nsnr + snr) * st.nstage + st.stage,
                 (size_t)st.nsnr * st.nstage, PERF ? 2 : 1, rl < st.rvalid);
}

template <int NPT>
static void launch_stage_fused_np(hipStream_t s, const SchemeK& sk, const StageArgs& st, const MmseK& mm, McBuffers& b,
                                  unsigned long long* counters, int rb) {
    const int ug = b.U / 64;
    uint16_t* qe_ = b.qe;
    uint16_t* qp_ = b.qp;
#define LAUNCH_SF(RBV)                                                                                          \
    {                                                                                                           \
        const int nrb = (sk.LK + 4 * (RBV) - 1) / (4 * (RBV));                                                  \
        if (st.mse_err) {                                                                                       \
            if (st.perfect)                                                                                     \
                hipLaunchKernelGGL((k_stage_fused<NPT, RBV, true, true>), dim3(ug * nrb), dim3(256), 0, s, sk, st, \
                                   nrb, mm.Wd, b.xp, b.sidx, b.h, b.hp, b.hest, qe_, qp_, b.v, b.u, counters); \
            else                                                                                                \
                hipLaunchKernelGGL((k_stage_fused<NPT, RBV, false, true>), dim3(ug * nrb), dim3(256), 0, s, sk,  \
                                   st, nrb, mm.Wd, b.xp, b.sidx, b.h, b.hp, b.hest, qe_, qp_, b.v, b.u,       \
                                   counters);                                                                   \
        } else if (st.perfect)                                                                                  \
            hipLaunchKernelGGL((k_stage_fused<NPT, RBV, true, false>), dim3(ug * nrb), dim3(256), 0, s, sk, st,   \
                               nrb, mm.Wd, b.xp, b.sidx, b.h, b.hp, b.hest, qe_, qp_, b.v, b.u, counters);     \
        else                                                                                                    \
            hipLaunchKernelGGL((k_stage_fused<NPT, RBV, false, false>), dim3(ug * nrb), dim3(256), 0, s, sk, st,  \
                               nrb, mm.Wd, b.xp, b.sidx, b.h, b.hp, b.hest, qe_, qp_, b.v, b.u, counters);     \
        return;                                                                                                 \
    }
    if (rb == 4) LAUNCH_SF(4)
    if (rb == 16) LAUNCH_SF(16)
    LAUNCH_SF(8)
#undef LAUNCH_SF
}

static bool stage_fused_ok(const Opts& op, const SchemeK& sk) {
    return !sk.despread && !op.stage_split && (sk.NP == 8 || sk.NP == 16 || sk.NP == 32) && sk.M <= 256 &&
           sk.nI <= 16 && sk.nQ <= 16;
}

bool perfect_fusable(const Opts& op, const SchemeK& sk) { return stage_fused_ok(op, sk) && sk.p_diag && op.pfuse; }

unsigned launch_stage(hipStream_t s, const Opts& op, const SchemeK& sk, const MmseK& mm, int stage, int var,
                      int n_iter, bool last, McBuffers& b, unsigned long long* counters, int scheme_index,
                      bool perfect) {
    StageArgs st;
    st.perfect = perfect ? 1 : 0;
    st.stage = stage;
    st.var = var;
    st.nsnr = mm.nsnr;
    st.nstage = n_iter + 1;
    st.scheme = scheme_index;
    st.last = last ? 1 : 0;
    st.tr = b.tr;
    st.R = b.R;
    st.rvalid = b.rvalid;
    st.U = b.U;
    st.snr0 = b.snr0;
    st.xcd_order = op.xcd;
    st.ysrc_e = stage == 0 ? b.y : b.yest;
    st.ysrc_p = stage == 0 ? b.y : b.yperf;
    st.mse_err = b.mse_err;
    st.mse_pow = b.mse_pow;
    const int rblk = (sk.LK + DSCE_RB - 1) / DSCE_RB;
    // select-mode schemes: k_ls + one fused pass (Opts::stage_split keeps the
    // 3-kernel path; Opts::stage_rb = rows per wave of the fused pass, 4 | 8 | 16)
    if (stage_fused_ok(op, sk)) {
        hipLaunchKernelGGL(k_ls, dim3(b.U / WAVE), dim3(WAVE), 0, s, sk, st, b.xp, b.hp);
        if (sk.NP == 8) launch_stage_fused_np<8>(s, sk, st, mm, b, counters, op.stage_rb);
        else if (sk.NP == 16) launch_stage_fused_np<16>(s, sk, st, mm, b, counters, op.stage_rb);
        else launch_stage_fused_np<32>(s, sk, st, mm, b, counters, op.stage_rb);
        if (!last && !sk.p_diag)
            hipLaunchKernelGGL(k_precode, dim3(b.U / WAVE, rblk), dim3(WAVE), 0, s, sk, st, b.xp, b.qe, b.qp, b.v,
                               b.u);
        return PATH_STAGE_FUSED;
    }
    hipLaunchKernelGGL(k_ls, dim3(b.U / WAVE), dim3(WAVE), 0, s, sk, st, b.xp, b.hp);
    hipLaunchKernelGGL(k_ls_hest, dim3(b.U / WAVE, rblk), dim3(WAVE), (size_t)sk.NP * WAVE * sizeof(double2), s, sk,
                       st, mm.Wd, b.h, b.hp, b.e, b.e2);
    hipLaunchKernelGGL(k_detect, dim3(b.U / WAVE, (sk.ND + DET_CHUNK - 1) / DET_CHUNK), dim3(WAVE), 0, s, sk, st,
                       b.sidx, b.e, b.e2, b.qe, b.qp, counters);
    if (!last)
        hipLaunchKernelGGL(k_precode, dim3(b.U / WAVE, rblk), dim3(WAVE), 0, s, sk, st, b.xp, b.qe, b.qp, b.v, b.u);
    return PATH_STAGE_SPLIT;
}

// MMSE one-tap channel h_hat = diag(D_hat) = sum_p W[(c,c),p] hP_p for n LS
// vectors (PSACE 'MMSE' slot, script:417-428); hp NP x n, h LK x n (column-major).
__global__ void k_mmse_onetap(int LK, int NP, const double2* __restrict__ wd, const double2* __restrict__ hp, int n,
                              double2* __restrict__ h) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int u = blockIdx.y;
    if (c >= LK || u >= n) return;
    double2 acc = make_double2(0.0, 0.0);
    for (int p = 0; p < NP; ++p) c_fma(acc, wd[(size_t)c * NP + p], hp[(size_t)u * NP + p]);
    h[(size_t)u * LK + c] = acc;
}

void launch_mmse_onetap(hipStream_t s, int LK, int NP, const double2* wd, const double2* hp, int n, double2* h) {
    hipLaunchKernelGGL(k_mmse_onetap, dim3((LK + 63) / 64, n), dim3(64), 0, s, LK, NP, wd, hp, n, h);
}

}  // namespace dsce
