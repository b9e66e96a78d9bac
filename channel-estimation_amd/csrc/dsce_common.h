// dsce_common.h — shared device/host definitions of the MI355X engine.
//
// Data layout in HBM: every per-realisation or
// per-unit vector is stored "structure of arrays", element-major with the
// realisation / unit index fastest ([element][unit]).  A wavefront maps its 64
// lanes to 64 units (unit = snr * R + rep), so every operator (G, Q, P, W) is
// wave-uniform and is read with scalar loads, while per-unit vectors are read
// and written with fully coalesced 16-byte lanes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DSCE_RB 24          // rows per block of the G / Q^H bands (banded matvec tile)
#define DSCE_WRB 32         // rows per block of the MMSE estimator W (two 16-row MFMA tiles)
#define DSCE_MAX_NP 64
#define DSCE_MAX_TAPS 64

// ---------------------------------------------------------------------------
// complex fp64 helpers (interleaved double2 = (re, im))
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ double2 c_make(double r, double i) { return make_double2(r, i); }
__host__ __device__ __forceinline__ double2 c_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__host__ __device__ __forceinline__ double2 c_sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__host__ __device__ __forceinline__ double2 c_mul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__host__ __device__ __forceinline__ double2 c_scale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
__host__ __device__ __forceinline__ double2 c_conj(double2 a) { return make_double2(a.x, -a.y); }
// a / b  (plain formula; rounding-level differences to numpy's Smith division)
__host__ __device__ __forceinline__ double2 c_div(double2 a, double2 b) {
    double d = b.x * b.x + b.y * b.y;
    return make_double2((a.x * b.x + a.y * b.y) / d, (a.y * b.x - a.x * b.y) / d);
}
// acc += a * b
__device__ __forceinline__ void c_fma(double2& acc, double2 a, double2 b) {
    acc.x = fma(a.x, b.x, acc.x);
    acc.x = fma(-a.y, b.y, acc.x);
    acc.y = fma(a.x, b.y, acc.y);
    acc.y = fma(a.y, b.x, acc.y);
}

// ---------------------------------------------------------------------------
// Philox4x32-10 and the random-stream spec of include/dsce.h
// ---------------------------------------------------------------------------
enum { STREAM_THETA = 1, STREAM_PHI = 2, STREAM_BITS = 3, STREAM_PILOTS = 4, STREAM_NOISE = 5 };

// a ^ b ^ c in one v_bitop3_b32 (gfx950; truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// rounds R0..9 of Philox4x32-10 on the state (c0..c3) with the round-R0 keys
template <int R0 = 0>
__device__ __forceinline__ uint4 philox_rounds(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                               uint32_t k1) {
#pragma unroll
    for (int r = R0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = xor3(hi1, c1, k0), n2 = xor3(hi0, c3, k1);
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
    return philox_rounds<0>(c0, c1, c2, c3, k0, k1);
}

__device__ __forceinline__ uint4 stream_block(uint64_t seed, uint64_t rep, uint32_t stream, uint32_t sub,
                                              uint32_t idx) {
    return philox4x32_10(idx, (uint32_t)rep, (uint32_t)(rep >> 32), ((stream & 0xFFFFu) << 16) | (sub & 0xFFFFu),
                         (uint32_t)seed, (uint32_t)(seed >> 32));
}

// stream_block of many sub-streams of one (seed, rep, stream, idx) (k_txrx_fft:
// the SNR points): the first round does not depend on the sub-stream except
// through one XOR (c2' = hi(M0 idx) ^ c3 ^ k1, with k1 = seed >> 32 the round-0
// key, not yet incremented), so its two products are formed once (pre) and each
// block costs nine rounds (tests/test_philox_sub.py restates the split)
struct PhiloxSub {
    uint32_t n0, lo1, hk, lo0, k0, k1;
};
__device__ __forceinline__ PhiloxSub stream_pre(uint64_t seed, uint64_t rep, uint32_t idx) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * idx, p1 = (uint64_t)0xCD9E8D57u * (uint32_t)(rep >> 32);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    return PhiloxSub{xor3((uint32_t)(p1 >> 32), (uint32_t)rep, k0), (uint32_t)p1, (uint32_t)(p0 >> 32) ^ k1,
                     (uint32_t)p0, k0 + 0x9E3779B9u, k1 + 0xBB67AE85u};
}
__device__ __forceinline__ uint4 stream_sub(const PhiloxSub& p, uint32_t stream, uint32_t sub) {
    return philox_rounds<1>(p.n0, p.lo1, p.hk ^ (((stream & 0xFFFFu) << 16) | (sub & 0xFFFFu)), p.lo0, p.k0, p.k1);
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// ---------------------------------------------------------------------------
// Banded block operator: rows grouped in blocks of <= DSCE_RB rows; every
// block has a contiguous reduction range [klo, khi) and its values are stored
// densely as vals[off + (k - klo) * DSCE_RB + r_local] (rows padded to RB with
// zeros).  Used for G (rows = samples, k = symbols), Q^H (rows = symbols,
// k = samples) and the MMSE estimator W (rows = symbols, k = (col, pilot)).
// ---------------------------------------------------------------------------
struct Band {
    int nblk;
    int rb;                       // row stride of the packed values (rows per block, padded)
    const int* row0;
    const int* nrows;
    const int* klo;
    const int* khi;
    const long long* off;
    const double2* vals;
};

// The MMSE estimator W as pair tiles for k_wpair3: per block the (row, column)
// pairs q = c_local * rbp + r (r fastest, rbp = 24 or 32 rows) in tiles of 16,
// each tile stored as [k-step][4 pilots][16 pairs] (one MFMA A operand per
// k-step, one 16-byte load per lane).  Element of (pair q, pilot p):
// vals[off + ((q/16) * nks + p/4) * 64 + (p%4) * 16 + q%16].
struct PairBand {
    int nblk, rbp, nks;
    const int* row0;
    const int* nrows;
    const int* clo;               // first column of the block
    const int* ntile;             // pair tiles (a multiple of 3 for rbp 24, of 2 for rbp 32)
    const long long* off;
};

// ---------------------------------------------------------------------------
// Scheme operators as seen by the Monte-Carlo kernels (all device pointers).
// ---------------------------------------------------------------------------
struct SchemeK {
    int N, LK, Nsym, NP, ND, M, mbits, despread, real_detect;
    int noise_slot;               // AWGN sub-stream group (include/dsce.h NOISE)
    int qh_disjoint;              // every sample lies in at most one Q^H row block's k-range
    double inv_sqrt_kappa, data_div;
    const int* pilot_pos;
    const int* data_pos;
    const int* considered;        // ND no-edge flags (int: uniform reads are scalar loads)
    const double2* symbols;       // M, sorted by bit label
    // nearest-neighbour slicer on the constellation grid
    int nI, nQ;
    const double* lvI;            // nI ascending real levels
    const double* lvQ;            // nQ ascending imag levels (nQ = 1, {0} for PAM)
    const int* grid_sym;          // nI * nQ -> symbol index
    double slI, slQ;              // 1 / level step (1 for a single level)
    double lv0I, lv0Q;            // lowest levels (host copies of lvI[0], lvQ[0])
    // precoder P (LK x Nsym) and P^H (Nsym x LK), CSR
    const int* p_ptr;
    const int* p_col;
    const double2* p_val;
    const int* ph_ptr;
    const int* ph_col;
    const double2* ph_val;
    Band G;                       // N x LK
    Band QH;                      // LK x N (conj(Q)^T)
    Band HD;                      // LK x (N * ntap): diag(Q'HG) coefficients, k = n * ntap + tau
    // perfect-CSI diag(D): Q columns compact (support start + QL values)
    const int* q_start;
    const double2* q_col;         // LK x QL
    int QL;
    const int* g_start;
    const double2* g_col;         // LK x GL
    int GL;
    // fused receiver stage (select-mode detection): per LK row the data-symbol
    // index detected there (-1: pilot / auxiliary); when P has at most one entry
    // per row and every data entry sits on its own row (p_diag, e.g. OFDM), the
    // entry's column (-1: none) and value, so re-precoding is row-local
    const int* row_data;          // LK
    const int* row_cons;          // LK: 1 if the row carries a considered (no-edge) data symbol
    const int* row_pcol;          // LK
    const double2* row_pval;      // LK
    int p_diag;
    // p_diag and every data row carries the same precoder value pv_data (r05:
    // the chain kernels stage the constellation pre-multiplied by it, so the
    // re-precoded decision is one LDS read instead of a complex product per row)
    int pv_uni;
    double2 pv_data;
    // p_diag and every pilot / data column sits on exactly one row: the TX
    // symbols can be drawn row by row in parallel (k_tx_rows)
    int tx_rows;
    // block-local perfect-CSI IC (pic_ok: every Q^H block's rows are the G
    // columns of its own samples, e.g. OFDM symbols; precondition of pf_ok)
    int pic_ok;
    // FFT form of the chain (k_pic_fft): every Q^H block is qs DFT24 over its
    // 24-sample window and every G block gs IDFT24 with a cyclic prefix >= the
    // max tap delay (checked entry by entry at pack time); pf_scale = qs gs
    int pf_ok;
    double2 pf_scale;
    double2 pf_gs, pf_qs;         // the two factors: G block = gs w^(l m), Q^H block = qs w^(-l m)
    // LDS tables of the chain kernels (pf_ok schemes), precomputed at
    // dsce_add_scheme (r06, build_chain_tables): a block's prologue copies entry
    // tid instead of deriving it from tid (the index arithmetic, twiddle lookups
    // and scale products were ~5 % of the chain kernels' VALU instructions)
    const double2* ct_symc;       // [256] stage_sym(symbol) * scI (k_pic_fft); 0 past M
    const double2* ct_sym;        // [256] stage_sym(symbol) (k_mic_pilot / k_mic_data); 0 past M
    const double2* ct_amt;        // [2][6][16] the matrix-core network's A_m (flat = the LDS order)
    const double2* ct_twa;        // [2][4][6] the DPP network's lane twiddles (flat = the LDS order)
    const unsigned* ct_grid;      // [64] slice6's byte grid [iI][iQ] (row stride 16) as words
    const double2* ct_rpv;        // [QH blk][24] row precoder value
    const int* ct_rdc;            // [QH blk][24] data index << 1 | no-edge, or -1
    const int* ct_rpc;            // [QH blk][24] pilot column of a pilot row, or -1
    const double2* ct_wrow;       // [QH blk][24] diag(D_hat) weight qs gs w^(-l) of a delayed tap
    // polyphase form (poly_ok, build_poly): with w = e^(2 pi i / L) and F = L,
    //   G[n, l + L k] = A_k[n] w^(l n) C[l][k],   Q^H[l + L k, n] = B_k[n] w^(-l n) E[l][k]
    // (A_k, B_k real windows), so G u = sum_k A_k IDFT(C u_k)(n mod F) and
    // (Q^H r)_k = E DFT(fold_k), fold_k[m] = sum_{n = m mod F} B_k[n] r[n]
    int poly_ok, poly_ni;         // poly_ni = ceil(N / F) <= POLY_NI
    int poly_F, poly_K;           // DFT size F = L, symbols K
    const double2* poly_C;        // [K][F]
    const double2* poly_E;        // [K][F]
    const double* poly_A;         // [F][K][POLY_NA]: A_k[m + F j] at j + 1 (0 at index 0 and outside [0, N))
    const double* poly_B;         // [F][K][POLY_NI]
    const double2* poly_tw;       // w^e, e = 0..F-1
};
constexpr int POLY_NI = 24;       // samples per residue class the polyphase kernels hold
constexpr int POLY_IH = POLY_NI / 2;   // ... per half (k_poly_chan block)
constexpr int POLY_NA = POLY_NI + 1;   // A table row: j = -1 .. POLY_NI - 1

struct ChannelK {
    int N, ntap;                  // ntap = number of non-zero taps
    int tap_delay[DSCE_MAX_TAPS];
    double sqrt_pdp[DSCE_MAX_TAPS];
    double fD, dt;                // fD == 0: time-invariant block fading (FastFading.m:241-246)
    int paths, model;             // model: 0 Jakes, 1 Uniform, 2 Discrete-Jakes, 3 Discrete-Uniform
    int nd;                       // discrete models: Doppler bins f = -nd..nd (FastFading.m:161)
    const double* sqrt_dspec;     // discrete models: sqrt(DiscreteDopplerSpectrum), 2 nd + 1 (device)
};

// host-side launch helpers (defined in the .hip translation units)
#define DSCE_HIP_CHECK(expr)                                                       \
    do {                                                                           \
        hipError_t _e = (expr);                                                    \
        if (_e != hipSuccess) throw dsce::HipError(_e, #expr, __FILE__, __LINE__); \
    } while (0)
