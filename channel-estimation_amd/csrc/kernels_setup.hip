// kernels_setup.hip — correlation matrices and the MMSE estimator
// (DoublySelectiveChannelEstimation.m:208-313, FastFading.m:321-407) on the GPU.
//
// R_vecH = E{vec(H) vec(H)^H} (FastFading.m:366-407) is never materialised:
// its only non-zeros couple H[a+tau, a] with H[b+tau, b] through
// PDPn[tau] * J0(2 pi fD dt (a-b)), so every product R_vecH * vec(V) collapses
// to a Toeplitz J0 matvec per tap ("m-coefficients" below).  Entries that the
// reference wraps into the next column for tau >= 2 (FastFading.m:377) multiply
// samples outside every pilot's support and are exactly zero for all
// configurations served here (pilot supports never touch sample 0 and N-1 at
// once); see DESIGN.md §Setup.
#include "dsce_kernels.h"

#include <stdlib.h>

#include <math.h>

namespace dsce {

// J0 lag table, FastFading.m:330-333: index lag + N - 1, lag in [-(N-1), N-1]
__global__ void k_time_correlation(int N, double fD, double dt, int model, double* tab) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * N - 1) return;
    const double t = dt * (double)(i - (N - 1));
    if (fD == 0.0) {                       // time-invariant channel: FastFading.m:338-339
        tab[i] = 1.0;
        return;
    }
    tab[i] = model == 0 ? j0(((M_PI * 2.0) * fD) * t) : (t == 0.0 ? 1.0 : sin(M_PI * (2.0 * fD * t)) / (M_PI * (2.0 * fD * t)));
}

void setup_time_correlation(hipStream_t s, int N, double fD, double dt, int model, double* j0tab) {
    hipLaunchKernelGGL(k_time_correlation, dim3((2 * N - 1 + 255) / 256), dim3(256), 0, s, N, fD, dt, model, j0tab);
}

// m[j][q][a] = PDPn[d_q] * sum_b J0(a-b) * Q[b+d_q, j] * conj(G[b, j])   (pilot j)
// i.e. reshape(R_vecH * kron(g_j.', q_j')', N, N) restricted to its band
// (script:213, :260).
__global__ void k_mcoef(SetupArgs a, const int* __restrict__ g_start, int GL, double2* __restrict__ m) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int jq = blockIdx.y;                   // pilot * ntap + q
    const int j = jq / a.ntap, q = jq % a.ntap;
    if (idx >= a.N) return;
    const int col = a.pilot_pos[j];
    const int d = a.tap_delay[q];
    const double pdp = a.pdp[q];
    const double2* __restrict__ Gc = a.G + (size_t)col * a.N;
    const double2* __restrict__ Qc = a.Q + (size_t)col * a.N;
    const int b0 = g_start[col];
    double2 acc = make_double2(0.0, 0.0);
    for (int b = b0; b < b0 + GL && b < a.N; ++b) {
        if (b + d >= a.N) break;
        const double2 g = Gc[b];
        const double2 qv = Qc[b + d];
        if ((g.x == 0.0 && g.y == 0.0) || (qv.x == 0.0 && qv.y == 0.0)) continue;
        const double2 w = c_mul(qv, c_conj(g));
        const double r = pdp * a.j0tab[idx - b + a.N - 1];
        acc.x += r * w.x;
        acc.y += r * w.y;
    }
    m[((size_t)j * a.ntap + q) * a.N + idx] = acc;
}

void setup_mcoef(hipStream_t s, const SetupArgs& a, const int* g_start, int GL, const int*, int, double2* m) {
    hipLaunchKernelGGL(k_mcoef, dim3((a.N + 255) / 256, a.NP * a.ntap), dim3(256), 0, s, a, g_start, GL, m);
}

// R_hP[i, j] = sum_n sum_q conj(Q[n+d_q, i]) m_j[q][n] G[n, i]   (script:212-215)
__global__ void k_rhp(SetupArgs a, const double2* __restrict__ m, double2* __restrict__ rhp) {
    const int i = blockIdx.x, j = blockIdx.y;
    __shared__ double2 part[256];
    const int ci = a.pilot_pos[i];
    const double2* __restrict__ Gc = a.G + (size_t)ci * a.N;
    const double2* __restrict__ Qc = a.Q + (size_t)ci * a.N;
    double2 acc = make_double2(0.0, 0.0);
    for (int n = threadIdx.x; n < a.N; n += blockDim.x) {
        const double2 g = Gc[n];
        if (g.x == 0.0 && g.y == 0.0) continue;
        for (int q = 0; q < a.ntap; ++q) {
            const int r = n + a.tap_delay[q];
            if (r >= a.N) continue;
            const double2 t = c_mul(c_conj(Qc[r]), m[((size_t)j * a.ntap + q) * a.N + n]);
            c_fma(acc, t, g);
        }
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) part[threadIdx.x] = c_add(part[threadIdx.x], part[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) rhp[(size_t)j * a.NP + i] = part[0];     // column-major NP x NP
}

void setup_rhp(hipStream_t s, const SetupArgs& a, const double2* m, double2* rhp) {
    hipLaunchKernelGGL(k_rhp, dim3(a.NP, a.NP), dim3(256), 0, s, a, m, rhp);
}

// Gp = G * P (script:203-205), dense N x Nsym column-major
__global__ void k_gp(SetupArgs a, double2* __restrict__ gp) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    if (n >= a.N) return;
    double2 acc = make_double2(0.0, 0.0);
    const double2* __restrict__ Pk = a.P + (size_t)k * a.LK;
    for (int c = 0; c < a.LK; ++c) {
        const double2 p = Pk[c];
        if (p.x == 0.0 && p.y == 0.0) continue;
        c_fma(acc, a.G[(size_t)c * a.N + n], p);
    }
    gp[(size_t)k * a.N + n] = acc;
}

void setup_gp(hipStream_t s, const SetupArgs& a, double2* gp) {
    hipLaunchKernelGGL(k_gp, dim3((a.N + 255) / 256, a.Nsym), dim3(256), 0, s, a, gp);
}

// Total received power at pilot i incl. interference of every precoded symbol
// (script:222-234):  |sum_{a,b} C_i[a,b] A[a,b]| with
// C_i[a,b] = sum_q PDPn conj(Q[a+d_q,i]) Q[b+d_q,i] J0(a-b) / kappa, A = Gp Gp^H.
__global__ void k_rest_diag(SetupArgs a, const double2* __restrict__ gp, const int* __restrict__ q_start, int QL,
                            double* __restrict__ diag) {
    const int i = blockIdx.x;
    const int ci = a.pilot_pos[i];
    const double2* __restrict__ Qc = a.Q + (size_t)ci * a.N;
    int maxd = 0;
    for (int q = 0; q < a.ntap; ++q) maxd = max(maxd, a.tap_delay[q]);
    const int s0 = max(0, q_start[ci] - maxd);
    const int s1 = min(a.N, q_start[ci] + QL);
    const int S = s1 - s0;
    __shared__ double2 part[256];
    double2 acc = make_double2(0.0, 0.0);
    for (int pr = threadIdx.x; pr < S * S; pr += blockDim.x) {
        const int aa = s0 + pr / S, bb = s0 + pr % S;
        double2 c = make_double2(0.0, 0.0);
        for (int q = 0; q < a.ntap; ++q) {
            const int ra = aa + a.tap_delay[q], rb = bb + a.tap_delay[q];
            if (ra >= a.N || rb >= a.N) continue;
            const double2 t = c_mul(c_conj(Qc[ra]), Qc[rb]);
            const double f = a.pdp[q] * a.j0tab[aa - bb + a.N - 1];
            c.x += f * t.x;
            c.y += f * t.y;
        }
        if (c.x == 0.0 && c.y == 0.0) continue;
        double2 A = make_double2(0.0, 0.0);
        for (int k = 0; k < a.Nsym; ++k)
            c_fma(A, gp[(size_t)k * a.N + aa], c_conj(gp[(size_t)k * a.N + bb]));
        c_fma(acc, c, A);
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) part[threadIdx.x] = c_add(part[threadIdx.x], part[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) diag[i] = hypot(part[0].x, part[0].y) / a.kappa;
}

void setup_rest_diag(hipStream_t s, const SetupArgs& a, const double2* gp, const int* q_start, int QL, double* diag) {
    hipLaunchKernelGGL(k_rest_diag, dim3(a.NP), dim3(256), 0, s, a, gp, q_start, QL, diag);
}

// pinv(R) for a Hermitian positive-definite NP x NP R: Gauss-Jordan with partial
// pivoting in LDS, one workgroup per matrix (script:283-285, :302-304).
__global__ void k_rinv(int NP, const double2* __restrict__ Rall, double2* __restrict__ Iall) {
    extern __shared__ double2 Aug[];          // NP x 2NP, row-major
    __shared__ int piv;
    const double2* R = Rall + (size_t)blockIdx.x * NP * NP;
    double2* Ri = Iall + (size_t)blockIdx.x * NP * NP;
    const int W2 = 2 * NP;
    for (int t = threadIdx.x; t < NP * W2; t += blockDim.x) {
        const int r = t / W2, c = t % W2;
        Aug[t] = c < NP ? R[(size_t)c * NP + r] : make_double2(c - NP == r ? 1.0 : 0.0, 0.0);
    }
    __syncthreads();
    for (int k = 0; k < NP; ++k) {
        if (threadIdx.x == 0) {
            int best = k;
            double bv = hypot(Aug[k * W2 + k].x, Aug[k * W2 + k].y);
            for (int r = k + 1; r < NP; ++r) {
                const double v = hypot(Aug[r * W2 + k].x, Aug[r * W2 + k].y);
                if (v > bv) { bv = v; best = r; }
            }
            piv = best;
        }
        __syncthreads();
        if (piv != k)
            for (int c = threadIdx.x; c < W2; c += blockDim.x) {
                const double2 t = Aug[k * W2 + c];
                Aug[k * W2 + c] = Aug[piv * W2 + c];
                Aug[piv * W2 + c] = t;
            }
        __syncthreads();
        const double2 d = Aug[k * W2 + k];
        __syncthreads();
        for (int c = threadIdx.x; c < W2; c += blockDim.x) Aug[k * W2 + c] = c_div(Aug[k * W2 + c], d);
        __syncthreads();
        for (int t = threadIdx.x; t < NP * W2; t += blockDim.x) {
            const int r = t / W2, c = t % W2;
            if (r == k) continue;
            const double2 f = Aug[r * W2 + k];
            if (c == k) continue;
            Aug[t] = c_sub(Aug[t], c_mul(f, Aug[k * W2 + c]));
        }
        __syncthreads();
        for (int r = threadIdx.x; r < NP; r += blockDim.x)
            if (r != k) Aug[r * W2 + k] = make_double2(0.0, 0.0);
        __syncthreads();
    }
    // one step of iterative refinement, X <- X + X (I - R X): brings the
    // Gauss-Jordan inverse to the accuracy the conditioning allows (the R_noI
    // of 32 pilots reaches cond ~1e5 at 36-40 dB)
    double2* E = Aug + (size_t)NP * W2;       // NP x NP, row-major
    for (int t = threadIdx.x; t < NP * NP; t += blockDim.x) {
        const int r = t / NP, c = t % NP;
        Aug[r * W2 + c] = R[(size_t)c * NP + r];  // left half <- R (row-major)
    }
    __syncthreads();
    for (int t = threadIdx.x; t < NP * NP; t += blockDim.x) {
        const int r = t / NP, c = t % NP;
        double2 acc = make_double2(r == c ? 1.0 : 0.0, 0.0);
        for (int k = 0; k < NP; ++k) acc = c_sub(acc, c_mul(Aug[r * W2 + k], Aug[k * W2 + NP + c]));
        E[t] = acc;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < NP * NP; t += blockDim.x) {
        const int r = t % NP, c = t / NP;        // column-major output
        double2 acc = make_double2(0.0, 0.0);
        for (int k = 0; k < NP; ++k) acc = c_add(acc, c_mul(Aug[r * W2 + NP + k], E[k * NP + c]));
        Ri[t] = c_add(Aug[r * W2 + NP + c], acc);
    }
}

void setup_rinv(hipStream_t s, int NP, int nmat, const double2* R, double2* Rinv) {
    hipLaunchKernelGGL(k_rinv, dim3(nmat), dim3(256), (size_t)NP * 3 * NP * sizeof(double2), s, NP, R, Rinv);
}

// The channel-estimate operator of the structured MMSE IC (k_mic_fft):
// D_hat = sum_p W_p hP_p = Q' H_hat G with H_hat = sum_p' M_p' z_p', z = pinv(R) hP
// (script:260, :283-285), so the estimated tap q at output sample n is
//   hhat[q][n] = sum_p bv[q][n][p] hP_p,  bv[q][n][p] = sum_p' m[p'][q][n - d_q] Rinv[p'][p]
// (m: k_mcoef's band of M_p', column n - d_q of the convolution matrix).
// grid (ceil(N NP / 256), ntap, nsl); Rinv column-major per slice.
__global__ void k_bv(SetupArgs a, const double2* __restrict__ m, const double2* __restrict__ rinv,
                     double2* __restrict__ bv) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int q = blockIdx.y, sl = blockIdx.z;
    if (e >= a.N * a.NP) return;
    const int n = e / a.NP, p = e % a.NP, b = n - a.tap_delay[q];
    const double2* __restrict__ ri = rinv + (size_t)sl * a.NP * a.NP + (size_t)p * a.NP;
    double2 acc = make_double2(0.0, 0.0);
    if (b >= 0)
        for (int pp = 0; pp < a.NP; ++pp) c_fma(acc, m[((size_t)pp * a.ntap + q) * a.N + b], ri[pp]);
    bv[(((size_t)sl * a.ntap + q) * a.N + n) * a.NP + p] = acc;
}

// bs[sl][blk][q][p] = sum_{j < win} bv[sl][q][klo[blk] + j][p]; one thread per entry
__global__ void k_bs(SetupArgs a, int nblk, const int* __restrict__ klo, int win, const double2* __restrict__ bv,
                     double2* __restrict__ bs) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int sl = blockIdx.y;
    if (e >= nblk * a.ntap * a.NP) return;
    const int p = e % a.NP, q = (e / a.NP) % a.ntap, blk = e / (a.NP * a.ntap);
    const double2* __restrict__ src = bv + (((size_t)sl * a.ntap + q) * a.N) * a.NP + p;
    double2 acc = make_double2(0.0, 0.0);
    for (int j = 0; j < win; ++j) {
        const int n = klo[blk] + j;
        if (n < a.N) acc = c_add(acc, src[(size_t)n * a.NP]);
    }
    bs[(size_t)sl * nblk * a.ntap * a.NP + e] = acc;
}

void setup_bv(hipStream_t s, const SetupArgs& a, int nsl, const double2* m, const double2* rinv, double2* bv,
              int nblk, const int* klo, int win, double2* bs) {
    hipLaunchKernelGGL(k_bv, dim3((a.N * a.NP + 255) / 256, a.ntap, nsl), dim3(256), 0, s, a, m, rinv, bv);
    hipLaunchKernelGGL(k_bs, dim3((nblk * a.ntap * a.NP + 255) / 256, nsl), dim3(256), 0, s, a, nblk, klo, win, bv, bs);
}

// R_Dij,hP column i = vec(Q' M_i G) with |.| < thr -> 0 (script:259-268), written
// straight into the packed band layout of W: off[blk] + ((c-c_lo)*NP + i)*RB + r.
__global__ void k_rdij(SetupArgs a, Band Wb, const double2* __restrict__ m, const int* __restrict__ g_start, int GL,
                       const int* __restrict__ q_start, int QL, double2* __restrict__ rd) {
    const int blk = blockIdx.x, i = blockIdx.y;
    const int row0 = Wb.row0[blk], nrows = Wb.nrows[blk];
    const int c_lo = Wb.klo[blk] / a.NP, c_hi = Wb.khi[blk] / a.NP;
    const int rb = Wb.rb;
    const int nslot = (c_hi - c_lo) * rb;
    double2* __restrict__ out = rd + Wb.off[blk];
    for (int t = threadIdx.x; t < nslot; t += blockDim.x) {
        const int c = c_lo + t / rb, rl = t % rb;
        double2 acc = make_double2(0.0, 0.0);
        if (rl < nrows) {
            const int r = row0 + rl;
            const double2* __restrict__ Qr = a.Q + (size_t)r * a.N;
            const double2* __restrict__ Gc = a.G + (size_t)c * a.N;
            const int gs = g_start[c];
            for (int n = q_start[r]; n < q_start[r] + QL && n < a.N; ++n) {
                const double2 qv = Qr[n];
                if (qv.x == 0.0 && qv.y == 0.0) continue;
                double2 mg = make_double2(0.0, 0.0);
                for (int q = 0; q < a.ntap; ++q) {
                    const int b = n - a.tap_delay[q];
                    if (b < gs || b >= gs + GL || b < 0) continue;
                    c_fma(mg, m[((size_t)i * a.ntap + q) * a.N + b], Gc[b]);
                }
                c_fma(acc, c_conj(qv), mg);
            }
            if (hypot(acc.x, acc.y) < a.thr) acc = make_double2(0.0, 0.0);
        }
        out[((size_t)(c - c_lo) * a.NP + i) * rb + rl] = acc;
    }
}

void setup_rdij(hipStream_t s, const SetupArgs& a, const Band& Wb, const double2* m, const int* g_start, int GL,
                const int* q_start, int QL, double2* rd) {
    hipLaunchKernelGGL(k_rdij, dim3(Wb.nblk, a.NP), dim3(256), 0, s, a, Wb, m, g_start, GL, q_start, QL, rd);
}

// W = R_Dij,hP * pinv(R) with |.| < thr -> 0 (script:283-289), packed layout;
// also extracts the diagonal W[(c,c),p] used for h_hat = diag(D_hat).
__global__ void k_w(SetupArgs a, Band Wb, const double2* __restrict__ rd, const double2* __restrict__ rinv,
                    double2* __restrict__ w, double2* __restrict__ wd) {
    const int blk = blockIdx.x;
    const int row0 = Wb.row0[blk], nrows = Wb.nrows[blk];
    const int c_lo = Wb.klo[blk] / a.NP, c_hi = Wb.khi[blk] / a.NP;
    const int rb = Wb.rb;
    const int nslot = (c_hi - c_lo) * rb;
    const double2* __restrict__ in = rd + Wb.off[blk];
    double2* __restrict__ out = w + Wb.off[blk];
    for (int t = threadIdx.x; t < nslot; t += blockDim.x) {
        const int cl = t / rb, rl = t % rb;
        const int c = c_lo + cl;
        for (int pp = 0; pp < a.NP; ++pp) {
            double2 acc = make_double2(0.0, 0.0);
            if (rl < nrows)
                for (int p = 0; p < a.NP; ++p)
                    c_fma(acc, in[((size_t)cl * a.NP + p) * rb + rl], rinv[(size_t)pp * a.NP + p]);
            if (hypot(acc.x, acc.y) < a.thr) acc = make_double2(0.0, 0.0);
            // the diagonal lives in wd only: the contraction applies D_hat - diag(D_hat)
            const bool dg = rl < nrows && row0 + rl == c;
            out[((size_t)cl * a.NP + pp) * rb + rl] = dg ? make_double2(0.0, 0.0) : acc;
            if (dg) wd[(size_t)c * a.NP + pp] = acc;
        }
    }
}

void setup_w(hipStream_t s, const SetupArgs& a, const Band& Wb, long long, const double2* rd, const double2* rinv,
             double2* w, double2* wd) {
    hipLaunchKernelGGL(k_w, dim3(Wb.nblk), dim3(256), 0, s, a, Wb, rd, rinv, w, wd);
}

}  // namespace dsce

namespace dsce {

// Non-zero column extent of every W block over all (variant, SNR) slices, after
// the 1e-8 threshold: lohi[2*blk] = min c_local, lohi[2*blk+1] = max c_local.
// The contraction skips exact zeros only, so trimming is bit-exact.
__global__ void k_w_extent(Band Wb, int NP, const double2* __restrict__ w, long long w_elems, int* __restrict__ lohi) {
    const int blk = blockIdx.x;
    const double2* __restrict__ ws = w + (size_t)blockIdx.y * w_elems + Wb.off[blk];
    const int ncol = (Wb.khi[blk] - Wb.klo[blk]) / NP;
    const long long n = (long long)ncol * NP * Wb.rb;
    int lo = 1 << 30, hi = -1;
    for (long long t = threadIdx.x; t < n; t += blockDim.x) {
        const double2 v = ws[t];
        if (v.x != 0.0 || v.y != 0.0) {
            const int c = (int)(t / ((long long)NP * Wb.rb));
            lo = min(lo, c);
            hi = max(hi, c);
        }
    }
    if (hi >= 0) {
        atomicMin(&lohi[2 * blk], lo);
        atomicMax(&lohi[2 * blk + 1], hi);
    }
}

void setup_w_extent(hipStream_t s, const Band& Wb, int NP, const double2* w, long long w_elems, int nslices, int* lohi) {
    hipLaunchKernelGGL(k_w_extent, dim3(Wb.nblk, nslices), dim3(256), 0, s, Wb, NP, w, w_elems, lohi);
}

// Pair-tile repack of the (trimmed, zero-diagonal) W band for k_wpair; rows past
// nrows and columns past the band's extent are zero.  grid (nblk, nslices).
__global__ void k_wpair_pack(Band Wb, int NP, const double2* __restrict__ w, long long w_elems, PairBand P,
                             double2* __restrict__ wp, long long wp_elems) {
    const int blk = blockIdx.x, sl = blockIdx.y;
    const double2* __restrict__ src = w + (size_t)sl * w_elems + Wb.off[blk];
    double2* __restrict__ dst = wp + (size_t)sl * wp_elems + P.off[blk];
    const int ncol = (Wb.khi[blk] - Wb.klo[blk]) / NP, nrows = Wb.nrows[blk];
    const long long n = (long long)P.ntile[blk] * P.nks * 64;
    for (long long e = threadIdx.x; e < n; e += blockDim.x) {
        const int t = (int)(e / (P.nks * 64)), rem = (int)(e % (P.nks * 64));
        const int ks = rem / 64, k4 = (rem % 64) / 16, i = rem % 16;
        const int q = 16 * t + i, cl = q / P.rbp, r = q % P.rbp, p = 4 * ks + k4;
        double2 v = make_double2(0.0, 0.0);
        if (r < nrows && cl < ncol && p < NP) v = src[((size_t)cl * NP + p) * Wb.rb + r];
        dst[e] = v;
    }
}

// 3M planes of the pair tiles: per (tile, k-step) the 64 lanes' Re, Im and
// Re+Im (k_wpair3's Gauss/Karatsuba form), the planes of two consecutive
// k-steps interleaved per lane, [tile][k-step pair][plane][lane][2], so
// k_wpair3 fetches them with 16-byte loads.  nks is even (2, 4 or 8).
__global__ void k_wpair_pack3(long long wp_elems, int nks, const double2* __restrict__ wp, double* __restrict__ w3) {
    const long long n = wp_elems;
    const double2* __restrict__ src = wp + (size_t)blockIdx.y * wp_elems;
    double* __restrict__ dst = w3 + (size_t)blockIdx.y * 3 * wp_elems;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
        const double2 v = src[e];
        const long long g = e / 64, l = e % 64;
        const double pv[3] = {v.x, v.y, v.x + v.y};
        const long long t = g / nks, ks = g % nks;
        for (int pl = 0; pl < 3; ++pl) dst[((t * (nks / 2) + ks / 2) * 3 + pl) * 128 + 2 * l + (ks & 1)] = pv[pl];
    }
}


// Operands of the fused MMSE stage (k_pilot_pre + k_wpair3<..., true>), block-
// diagonal schemes only.  Wpil[slice][pilot i][cc][p] = W[(pilot row, c0_i + cc), p]
// from the packed band (the pilot rows of W, row-major: the pre-pass streams
// them with wave-uniform loads); c0_i = first column of the pilot row's block.
__global__ void k_wpil_pack(Band Wb, int NP, const double2* __restrict__ w, long long w_elems,
                            const int* __restrict__ pil_blk, const int* __restrict__ pilot_pos, int ncol,
                            double2* __restrict__ out) {
    const int i = blockIdx.x, sl = blockIdx.y;
    const int b = pil_blk[i], r = pilot_pos[i];
    const int clo = Wb.klo[b] / NP, chi = Wb.khi[b] / NP;
    const int c0 = Wb.row0[b];
    for (int e = threadIdx.x; e < ncol * NP; e += blockDim.x) {
        const int cc = e / NP, p = e % NP, c = c0 + cc;
        double2 v = make_double2(0.0, 0.0);
        if (c >= clo && c < chi)
            v = w[(size_t)sl * w_elems + Wb.off[b] + ((size_t)(c - clo) * NP + p) * Wb.rb + (r - Wb.row0[b])];
        out[(((size_t)sl * NP + i) * ncol + cc) * NP + p] = v;
    }
}

// WdA[slice][blk][t][ks][lane] = Wd[slice][row0_blk + 16 t + (lane & 15)][4 ks + (lane >> 4)]:
// diag(W) rows as the A operand of v_mfma_f64_16x16x4 (diag(D_hat) = Wd hP on the matrix cores)
__global__ void k_wda_pack(Band Wb, int LK, int NP, const double2* __restrict__ wd, double2* __restrict__ out) {
    const int b = blockIdx.x, sl = blockIdx.y, nks = NP / 4;
    const int row0 = Wb.row0[b], nrows = Wb.nrows[b];
    for (int e = threadIdx.x; e < 2 * nks * 64; e += blockDim.x) {
        const int l = e & 63, ks = (e >> 6) % nks, t = (e >> 6) / nks;
        const int r = 16 * t + (l & 15);
        const double2 v = r < nrows ? wd[(size_t)sl * LK * NP + (size_t)(row0 + r) * NP + 4 * ks + (l >> 4)]
                                    : make_double2(0.0, 0.0);
        out[((size_t)sl * Wb.nblk + b) * 2 * nks * 64 + e] = v;
    }
}

void setup_fused_stage(hipStream_t s, const Band& Wb, int LK, int NP, const double2* w, long long w_elems,
                       const double2* wd, int nslices, const int* pil_blk, const int* pilot_pos, int ncol,
                       double2* wpil, double2* wda) {
    hipLaunchKernelGGL(k_wpil_pack, dim3(NP, nslices), dim3(256), 0, s, Wb, NP, w, w_elems, pil_blk, pilot_pos, ncol,
                       wpil);
    hipLaunchKernelGGL(k_wda_pack, dim3(Wb.nblk, nslices), dim3(256), 0, s, Wb, LK, NP, wd, wda);
}

void setup_wpair(hipStream_t s, const Band& Wb, int NP, const double2* w, long long w_elems, const PairBand& P,
                 double2* wp, long long wp_elems, int nslices, double* w3) {
    hipLaunchKernelGGL(k_wpair_pack, dim3(Wb.nblk, nslices), dim3(256), 0, s, Wb, NP, w, w_elems, P, wp, wp_elems);
    if (w3) hipLaunchKernelGGL(k_wpair_pack3, dim3(256, nslices), dim3(256), 0, s, wp_elems, P.nks, wp, w3);
}

// ---------------------------------------------------------------------------
// D = Q^H H G of one realisation (dsce_transmission_matrix, the parity probe of
// SURVEY §8(b); script:381-393, H = GetConvolutionMatrix{1}, FastFading.m:276-295:
// H[n, n - d_q] = IR_q[n] for n >= d_q).  Two passes over the dense operators:
// HG[n][c] = sum_q IR_q[n] G[n - d_q][c], then D[r][c] = sum_n conj(Q[n][r])
// HG[n][c] over Q column r's support [qlo[r], qhi[r]).  Test-only: the hot path
// never forms D (diag(D) and D u only).
// ---------------------------------------------------------------------------
__global__ void k_hg(ChannelK ch, int LK, const double2* __restrict__ ir, int R, int lane,
                     const double2* __restrict__ G, double2* __restrict__ hg) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)ch.N * LK) return;
    const int n = (int)(i % ch.N);
    const size_t c = i / ch.N;
    double2 acc = make_double2(0.0, 0.0);
    for (int q = 0; q < ch.ntap; ++q) {
        const int m = n - ch.tap_delay[q];
        if (m >= 0) c_fma(acc, ir[((size_t)q * ch.N + n) * R + lane], G[c * ch.N + m]);
    }
    hg[i] = acc;
}

__global__ void k_qh_hg(int N, int LK, const double2* __restrict__ Q, const int* __restrict__ qlo,
                        const int* __restrict__ qhi, const double2* __restrict__ hg, double2* __restrict__ D) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)LK * LK) return;
    const int r = (int)(i % LK);
    const size_t c = i / LK;
    double2 acc = make_double2(0.0, 0.0);
    for (int n = qlo[r]; n < qhi[r]; ++n) {
        const double2 q = Q[(size_t)r * N + n], h = hg[c * N + n];
        acc.x = fma(q.x, h.x, fma(q.y, h.y, acc.x));          // conj(q) h
        acc.y = fma(q.x, h.y, fma(-q.y, h.x, acc.y));
    }
    D[i] = acc;
}

void setup_transmission_matrix(hipStream_t s, const ChannelK& ch, int LK, const double2* ir, int R, int lane,
                               const double2* G, const double2* Q, const int* qlo, const int* qhi, double2* hg,
                               double2* D) {
    const size_t nhg = (size_t)ch.N * LK, nd = (size_t)LK * LK;
    hipLaunchKernelGGL(k_hg, dim3((unsigned)((nhg + 255) / 256)), dim3(256), 0, s, ch, LK, ir, R, lane, G, hg);
    hipLaunchKernelGGL(k_qh_hg, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, ch.N, LK, Q, qlo, qhi, hg, D);
}

// G[n, l + L k] in closed form (OFDM.m:153-165, :184-203; FBMC.m:255-285,
// :318-342) and Q = G * rx_scale with OFDM cyclic-prefix samples zeroed
// (OFDM.m:205-218).  The IFFT of a unit impulse at bin b is
// exp(j 2 pi b j / FFT) / FFT; the phase is reduced exactly in integers.
__global__ void k_tx_matrix(TxDesc d, const double* __restrict__ proto, double2* __restrict__ G,
                            double2* __restrict__ Q) {
    const long long LK = (long long)d.L * d.K;
    const long long total = LK * d.N;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(e % d.N), col = (int)(e / d.N);
        const int l = col % d.L, k = col / d.L;
        double2 g = make_double2(0.0, 0.0);
        bool cp = false;
        if (d.kind == 0) {                                   // OFDM
            const int m = n - d.zg - k * d.ts;
            const int body = d.ts - d.cp;                    // = FFT size
            if (m >= 0 && m < d.ts) {
                const int j = m >= d.cp ? m - d.cp : body - d.cp + m;
                cp = m < d.cp;
                const long long ph = ((long long)(l + d.ifb) * j) % d.fft;
                double sn, cs;
                sincospi(2.0 * (double)ph / (double)d.fft, &sn, &cs);
                const double a = d.norm / (double)d.fft;
                g = make_double2(a * cs, a * sn);
            }
        } else {                                             // FBMC Hermite-OQAM
            int np_ = n - k * d.ts;
            np_ %= d.N;
            if (np_ < 0) np_ += d.N;                         // np.roll is circular
            if (np_ < d.proto) {
                const int row = (l + d.ifb) % d.fft;
                const long long ph = ((long long)row * (np_ % d.fft)) % d.fft;
                double sn, cs;
                sincospi(2.0 * (double)ph / (double)d.fft, &sn, &cs);
                // PhaseShift[l, 0] = exp(j pi/2 l) exp(j phase0); times j^k (FBMC.m:336)
                double ps, pc;
                sincos(0.5 * M_PI * (double)((l + k) & 3) + d.phase0, &ps, &pc);
                const double a = proto[np_] * d.norm / (double)d.fft;
                const double2 e1 = make_double2(cs, sn), e2 = make_double2(pc, ps);
                g = make_double2(a * (e1.x * e2.x - e1.y * e2.y), a * (e1.x * e2.y + e1.y * e2.x));
            }
        }
        if (G) G[e] = g;
        if (Q) Q[e] = cp ? make_double2(0.0, 0.0) : make_double2(g.x * d.rx_scale, g.y * d.rx_scale);
    }
}

void setup_tx_matrix(hipStream_t s, const TxDesc& d, const double* proto, double2* G, double2* Q) {
    hipLaunchKernelGGL(k_tx_matrix, dim3(4096), dim3(256), 0, s, d, proto, G, Q);
}

}  // namespace dsce

namespace dsce {

// ---------------------------------------------------------------------------
// Measured FP64 matrix-core peak (the roofline denominator next to the 78.6 TF
// spec, which the microarchitecture guide does not list as measured): every
// wave issues back-to-back v_mfma_f64_16x16x4_f64 on NACC independent
// accumulators (no dependent-latency stalls), 2048 flops each.
// ---------------------------------------------------------------------------
typedef double pk4 __attribute__((ext_vector_type(4)));
static constexpr int PEAK_NACC = PEAK_MFMA_PER_ITER;

__global__ void __launch_bounds__(256) k_mfma_f64_peak(int iters, double seed, double* __restrict__ out) {
    pk4 acc[PEAK_NACC];
#pragma unroll
    for (int k = 0; k < PEAK_NACC; ++k) acc[k] = (pk4){0.0, 0.0, 0.0, 0.0};
    const double a = seed + 1e-3 * (threadIdx.x & 63), b = 1.0 - 1e-3 * (threadIdx.x & 7);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < PEAK_NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PEAK_NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

void launch_mfma_f64_peak(hipStream_t s, int blocks, int iters, double* out) {
    hipLaunchKernelGGL(k_mfma_f64_peak, dim3(blocks), dim3(256), 0, s, iters, 0.5, out);
}

}  // namespace dsce
