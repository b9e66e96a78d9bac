// dsce_kernels.h — host-callable launchers of the HIP kernels.
#pragma once

#include "dsce_common.h"

#include <vector>

namespace dsce {

// Kernel-selection options of a context (dsce_set_option; defaults = the
// measured-best path).  Read by the launchers; nothing reads the environment.
struct Opts {
    int xcd = 1;              // XCD-aware work order (each XCD walks a contiguous range)
    int fuse_stage = 1;       // MMSE stage of the IC iterations fused into the contraction
    int pic_chain = 3;        // perfect-CSI IC: 0 per-iteration passes, 1 VALU chain, 2 MFMA chain, 3 FFT chain
    int pfuse = 1;            // perfect-CSI detection fused into the second banded pass
    int stage_split = 0;      // 1: 3-kernel stage (k_ls_hest, k_detect, k_precode) for every scheme
    int stage_rb = 8;         // rows per wave of k_stage_fused: 4 | 8 | 16
    int noise_fuse = 1;       // AWGN drawn inside the Q^H pass (disjoint Q^H blocks)
    int snr_chunk = 0;        // SNR points per receiver chunk (0: all)
    int jakes_rpw = 2;        // realisations per Jakes wave (1 | 2)
    int wtrim = 1;            // trim W to its non-zero column extent (read by dsce_build_mmse)
    int wcontract_valu = 0;   // 1: VALU contraction instead of the MFMA pair tiles
    int mmse_ic = 1;          // MMSE branch of FFT-form OFDM as Q' H_hat G (k_mic_pilot + k_mic_data); 0: W contraction
    int jakes_win = 1;        // Jakes taps only at the samples some Q^H row reads (JakesChunks)
    int txrx_fft = 1;         // TX + channel + receiver front of FFT-form OFDM in one pass (k_txrx_fft)
    int snr_base = 0;         // noise sub-stream of SNR index k is snr_base + k (SNR-sharded sweeps)
    int tx_rows = 1;          // row-local precoders: TX symbols drawn row-parallel (k_tx_rows)
    int pic_net = 1;          // k_pic_fft's 4-point network: 1 = v_mfma_f64_4x4x4 (quarters on 16-lane rows), 0 = DPP
    int mic_net = 3;          // the same network for k_mic_data (bit 0) / k_mic_pilot (bit 1), whose tap GEMM then
                              // needs no exchange: data 3.99 -> 3.65 ms, pilot 1.91 -> 2.00 ms (237 VGPRs, r03: 1);
                              // with the low-rank taps the pilot kernel gains too: 1.625 -> 1.576 ms (r04: 3)
    int realise_win = 0;      // dsce_channel_realise forms only the JakesChunks samples (tests the window kernels)
    int mic_lr = 1;           // MMSE IC taps in the low-rank form T_k Z (k_mic_pilot / k_mic_data) where
                              // build_mic_lr verified it; 0 = the tap GEMM Bv hP on the matrix cores
    int pic_poly = 1;         // perfect-CSI IC passes of polyphase schemes (SchemeK::poly_ok: FBMC, OFDM with
                              // L != 24) as IDFT-L per symbol + window sums per residue + DFT-L per symbol
                              // (k_poly_syn / k_poly_chan / k_poly_ana) instead of the two banded passes
                              // (r04 box, C3: 14.3 -> 8.7 ms per iteration); 0 = the banded passes
    int wrow = 1;             // unfused W contraction of 32-row blocks (FBMC, C5) as one GEMM per row tile
                              // (k_wrow3: X = hP v_c as the B operand, no per-tile epilogue); 0 = k_wpair3
    int jakes_grp2 = 1;       // two-tap channels: k_jakes_grp2 (both taps per wave, each Philox block drawn
                              // once, LG = 16 / anchor groups); 0 = k_jakes_grp per tap
    int jakes_mom = 2;        // Jakes taps of the read windows: 2 = Taylor anchors over groups of windows
                              // (k_jakes_grp), 1 = one anchor per window (k_jakes_mom), 0 = recurrence;
                              // each where its truncation is below rounding, else the next lower
};

// Kernels a scheme's last dsce_run / dsce_trace_unit_ex went through
// (dsce_path_info; bit values mirrored in include/dsce.h DSCE_PATH_*).
enum : unsigned {
    PATH_WPAIR3_FUSED = 1u << 0,   // k_pilot_pre + k_wpair3<.., FUSE> (stage in the contraction epilogue)
    PATH_WPAIR3 = 1u << 1,         // k_wpair3 (3M, unfused)
    PATH_WPAIR4M = 1u << 2,        // retired (r01-r02 k_wpair, 4 real MFMAs per complex product)
    PATH_WCONTRACT_VALU = 1u << 3, // k_wcontract_valu
    PATH_PIC_MFMA = 1u << 4,       // k_pic_mfma (perfect-CSI chain on the matrix cores)
    PATH_PIC_CHAIN = 1u << 5,      // k_pic_chain (VALU chain)
    PATH_PIC_PASSES = 1u << 6,     // G u pass + Q^H H pass per iteration
    PATH_STAGE_FUSED = 1u << 7,    // k_ls + k_stage_fused
    PATH_STAGE_SPLIT = 1u << 8,    // k_ls_hest + k_detect + k_precode
    PATH_NOISE_FUSED = 1u << 9,    // noise drawn inside the Q^H pass
    PATH_PIC_FFT = 1u << 10,       // k_pic_fft (perfect-CSI chain by FFT, OFDM)
    PATH_MIC_FFT = 1u << 11,       // MMSE IC as Q' H_hat G by FFT (OFDM; k_mic_pilot + k_mic_data)
    PATH_TXRX_FFT = 1u << 12,      // k_txrx_fft (TX + channel + noisy receiver front by FFT, OFDM)
    PATH_PILOT_FUSED = 1u << 13,   // retired (r02 k_mic_fft's fused pilot pass)
    PATH_MIC_STAGES = 1u << 14,    // k_mic_pilot + k_mic_data: every MMSE stage in one launch pair
    PATH_MIC_LR = 1u << 15,        // ... with the low-rank tap operator T_k Z (build_mic_lr)
    PATH_PIC_POLY = 1u << 16,      // perfect-CSI IC by polyphase synthesis / analysis (k_poly_*)
    PATH_WROW3 = 1u << 17,         // unfused W contraction as one GEMM per row tile (k_wrow3)
};

// Per-stage trace of one unit (dsce_trace_unit_ex): every kernel that forms one
// of these quantities for unit `unit` of the traced scheme writes it here.
// Device arrays, stage-major: [stage][LK] / [stage][ND].
struct TraceK {
    int unit;
    int LK, ND;
    double2* yest;     // y_est of stage s (the MMSE IC input y - (D_hat - diag) v), s >= 1
    double2* yperf;    // y_perf of stage s (perfect-CSI IC), s >= 1
    double2* hest;     // diag(D_hat) of stage s
    int* dec_e;        // detected symbol index per data symbol, MMSE branch
    int* dec_p;        // perfect-CSI branch
};

struct McBuffers {
    int R;            // repetitions per batch (multiple of 64)
    int rvalid;       // the first rvalid of them count (a tail batch of a run whose
                      // length is no multiple of 64 pads the last wave; the padding
                      // realisations are simulated but add nothing to any counter)
    int nsnr;
    int U;            // units of the current SNR chunk = nchunk * R, unit = (snr - snr0) * R + rep
    int snr0;         // first SNR index of the chunk being processed
    // per repetition (channel shared by all schemes)
    double2* ir;      // [ntap][N][R]
    // per repetition and scheme
    double2* xp;      // [NP][R]
    uint16_t* sidx;   // [ND][R]
    double2* r0;      // [N][R]
    double2* h;       // [LK][R]   perfect-CSI diag(D)
    double2* xs;      // [LK][R]   scratch: precoded symbols
    double2* ss;      // [N][R]    scratch: time signal
    // per unit
    double2* y;       // [LK][U]
    double2* yest;    // [LK][U]
    double2* yperf;   // [LK][U]
    double2* hp;      // [NP][U]   LS pilot estimates of the current stage
    double2* hp2;     // [NP][U]   second buffer (fused MMSE stage: previous / current stage)
    double2* hest;    // [LK][U]   diag(D_hat) of the current stage
    double2* v;       // [LK][U]   P [xP; Q(x_est)]
    double2* u;       // [LK][U]   P [xP; Q(x_perfect)]
    double2* t;       // [N][U]    scratch: r / G u
    double2* e;       // [LK][U]   y_est ./ h_hat (one-tap quotient, MMSE)
    double2* e2;      // [LK][U]   y_perf ./ h     (one-tap quotient, perfect CSI)
    uint16_t* qe;     // [ND][U]   quantised symbol indices (estimate)
    uint16_t* qp;     // [ND][U]   quantised symbol indices (perfect CSI)
    uint16_t* sidr;   // [LK][R]   transmitted symbol index per data row (row-indexed sidx)
    double2* hpa;     // [stage][NP][U] LS pilot estimates of every stage (k_mic_pilot -> k_mic_data), or null
    int hpa_stages;   // stages hpa holds
    double2* za;      // [stage][ntap * MIC_NB][U] Z = Bz hP of every stage (low-rank MMSE IC), or null
    double2* pv;      // [LK][U] polyphase IC: IDFT of each symbol's C u (k_poly_syn), or null
    double2* pf;      // [LK][U] polyphase IC: window sums of r0 per (symbol, residue), first half (k_poly_chan)
    double2* pf2;     // [LK][U] ... second half; pv / pf / pf2 null unless Opts::pic_poly and a scheme has the form
    double* mse_err;  // null, or [scheme][snr][stage] sums of |h_hat - h|^2 (dsce_enable_mse)
    double* mse_pow;  // [scheme][snr] sums of |h|^2
    const TraceK* tr; // device trace of one unit (null: not tracing this scheme / chunk)
};

struct MmseK {
    const double2* W;     // [var][snr][w_elems] packed band layout
    const double2* Wd;    // [var][snr][LK][NP] diagonal entries W[(c,c),p]
    long long w_elems;
    int nsnr;
    Band Wb;              // block geometry (vals unused; per-(var,snr) base added)
    const double* Wp3;    // [var][snr][3 wp_elems] Re / Im / Re+Im planes (3M form), or null
    long long wp_elems;
    PairBand Pb;
    // fused MMSE stage (block-diagonal W, row-local P): null when not eligible
    const double2* Wpil;  // [var][snr][NP pilots][24 columns][NP]
    const double2* WdA;   // [var][snr][blk][2][NP/4][64] diag(W) rows, MFMA A layout
    const int* pil_c0;    // NP: first column of each pilot row's block
    // structured MMSE IC (k_mic_pilot / k_mic_data): H_hat taps = Bv hP; null when not eligible
    const double2* Bv;    // [var][snr][ntap][N][NP]
    const double2* Bs;    // [var][snr][QH blk][ntap][NP]: Bv summed over each block's FFT window
    const int* pblk;      // QH blocks holding pilot rows (k_pilot_fft)
    int npb;
    const int* dblk;      // QH blocks without pilot rows (k_mic_data)
    int ndb;
    const int* pmask;     // [QH blk]: 1 = holds pilot rows
    // the low-rank form of Bv (build_mic_lr): bv[q][n][p] = sum_k T_k[n] Bz[q k][p],
    // T_k the J0 kernel summed over pilot symbol k's FFT window; null when not eligible
    const double2* Bz;    // [var][snr][ntap * MIC_NB][NP]
    const double* Tw;     // [QH blk][MIC_NB][24]: T_k over the block's FFT window
    const double* Ts;     // [QH blk][MIC_NB]: its window sums
};
// pilot symbols (FFT windows holding pilots) of the low-rank MMSE IC operator
constexpr int MIC_NB = 4;

// Monte-Carlo pipeline.  Launchers return the PATH_* bits of the kernels they ran.
// Chunks of the impulse response a batch needs: every sample some Q^H row of
// some scheme reads (the channel taps are used at output samples only there:
// r0 = H s, diag(D) and the perfect-CSI passes / chains all go through Q^H).
struct JakesChunks {
    static constexpr int LEN = 24;   // samples per chunk
    const int* n0 = nullptr;         // device: first sample of each chunk
    int n = 0;
    std::vector<int> n0h;            // host copy of n0 (the anchor grouping)
    // k_jakes_grp anchor groups (jakes_grouping): runs of consecutive chunks whose
    // span keeps |theta k| <= JAKES_XMAX around the group centre; grp[g] =
    // (first chunk, chunk count); lg lanes per group, mt Taylor terms.  Rebuilt
    // when theta = 2 pi |fD| dt changes; ngrp == 0: not usable.
    const int2* grp = nullptr;
    int ngrp = 0, lg = 0, mt = 0;
    double theta = -1.0;
    int nsch_grp = -1;               // chunk count the groups were built for
};
// the anchor groups' limit: |theta k| <= JAKES_XMAX (the Taylor sum's terms grow
// to e^x / sqrt(2 pi x) before they fall: x = 3 costs ~20x the per-term rounding)
constexpr double JAKES_XMAX = 3.0;
// jc: form only those chunks (samples outside stay as they are: zero).  Returns
// which kernel ran (the work model of dsce_kernel_work): JAKES_KIND_GRP
// k_jakes_grp, JAKES_KIND_MOM k_jakes_mom, else JAKES_KIND_OTHER.
enum { JAKES_KIND_OTHER = 0, JAKES_KIND_MOM = 2, JAKES_KIND_GRP = 3 };
int launch_jakes(hipStream_t s, const Opts& op, const ChannelK& ch, uint64_t seed, uint64_t rep0, int R,
                  double2* ir, const JakesChunks* jc = nullptr);
// txrx (txrx_fft_ok): only the symbols; k_txrx_fft forms s, r0 and diag(D) in
// launch_rx_front
void launch_tx(hipStream_t s, const SchemeK& sk, const ChannelK& ch, int bits_slot, int pilot_slot, uint64_t seed,
               uint64_t rep0, McBuffers& b, bool txrx = false, bool rows = true);
bool txrx_fft_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b);
unsigned launch_rx_front(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, const double* pn,
                         uint64_t seed, uint64_t rep0, McBuffers& b);
unsigned launch_stage(hipStream_t s, const Opts& op, const SchemeK& sk, const MmseK& mm, int stage, int var,
                      int n_iter, bool last, McBuffers& b, unsigned long long* counters, int scheme_index,
                      bool perfect);
// true when launch_stage uses the fused select-mode pass and the precoder is
// row-local, so the perfect-CSI branch of IC iterations can ride on perfect_ic
bool perfect_fusable(const Opts& op, const SchemeK& sk);
unsigned launch_wcontract(hipStream_t s, const Opts& op, const SchemeK& sk, const MmseK& mm, int var, McBuffers& b);
// Fused MMSE stage of IC iteration `stage` (block-diagonal W, row-local P):
// k_pilot_pre (pilot rows + LS into hp_new) then the contraction with the
// stage's detection in its epilogue (no y_est, no separate stage kernel).
bool mmse_fused_ok(const Opts& op, const SchemeK& sk, const MmseK& mm, const McBuffers& b);
void launch_pilot_pre(hipStream_t s, const SchemeK& sk, const MmseK& mm, int var_prev, McBuffers& b,
                      const double2* hp_prev, double2* hp_new);
unsigned launch_mmse_fused(hipStream_t s, const Opts& op, const SchemeK& sk, const MmseK& mm, int var_prev,
                           int var_cur, int stage, int n_iter, bool last, McBuffers& b, const double2* hp_prev,
                           double2* hp_new, unsigned long long* counters, int scheme_index);
// Perfect-CSI detection fused into the perfect IC pass (select mode, row-local P)
struct PerfectDetectArgs {
    unsigned long long* counters;
    int scheme, stage, nstage, nsnr, last;
    double sI, sQ;   // 1 / slicer step (I, Q)
};
// Every MMSE stage (0..n_iter) of an FFT-form OFDM scheme: k_mic_pilot +
// k_mic_data, y_ic = y - Q'(H_hat (G v)) + diag(D_hat) v by the DFT-24 chain;
// the perfect-CSI branch then runs k_pic_fft with its stage 0
bool mmse_stages_ok(const Opts& op, const SchemeK& sk, const MmseK& mm, const ChannelK& ch, const McBuffers& b,
                    int niter);
// part: 1 = k_mic_pilot, 2 = k_mic_data (the data kernel reads the pilot kernel's hpa)
unsigned launch_mmse_stages(hipStream_t s, const SchemeK& sk, const MmseK& mm, const ChannelK& ch, McBuffers& b,
                            const PerfectDetectArgs* pd, int niter, int xcd, int part, bool nm = true, bool lr = false);
unsigned launch_perfect_ic(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, McBuffers& b,
                           const PerfectDetectArgs* pd);
// The whole perfect-CSI IC chain (iterations 1..niter) in one kernel, u in
// registers (pic_ok schemes); perfect_chain_ok tells when it applies.
bool perfect_chain_ok(const Opts& op, const SchemeK& sk, const ChannelK& ch, const McBuffers& b, int niter);
// stage0: k_pic_fft also runs the perfect-CSI stage 0 (one-tap y ./ h) first
unsigned launch_perfect_chain(hipStream_t s, const Opts& op, const SchemeK& sk, const ChannelK& ch, McBuffers& b,
                              const PerfectDetectArgs* pd, int niter, bool stage0 = false);
void launch_mmse_onetap(hipStream_t s, int LK, int NP, const double2* wd, const double2* hp, int n, double2* h);

// setup (correlation matrices and MMSE estimator)
struct SetupArgs {
    int N, LK, NP, Nsym, ntap, nsnr;
    const int* pilot_pos;
    const double2* G;        // dense N x LK (column-major)
    const double2* Q;        // dense N x LK
    const double2* P;        // dense LK x Nsym
    const double* j0tab;     // 2N-1 time correlation, index lag + N - 1
    int tap_delay[DSCE_MAX_TAPS];
    double pdp[DSCE_MAX_TAPS];
    double kappa;
    const double* pn;        // nsnr
    double thr;
};

void setup_time_correlation(hipStream_t s, int N, double fD, double dt, int model, double* j0tab);
void setup_mcoef(hipStream_t s, const SetupArgs& a, const int* g_start, int GL, const int* q_start, int QL,
                 double2* m /* [NP][ntap][N] */);
void setup_rhp(hipStream_t s, const SetupArgs& a, const double2* m, double2* rhp);
void setup_gp(hipStream_t s, const SetupArgs& a, double2* gp /* N x Nsym */);
void setup_rest_diag(hipStream_t s, const SetupArgs& a, const double2* gp, const int* q_start, int QL, double* diag);
void setup_rinv(hipStream_t s, int NP, int nmat, const double2* R, double2* Rinv);
// H_hat operator of the structured MMSE IC: bv[sl][q][n][p] = sum_p' m[p'][q][n - d_q]
// Rinv_sl[p'][p] for the nsl = 2 nsnr inverses; bs[sl][blk][q][p] = its sums over
// the FFT windows [klo[blk], klo[blk] + win)
void setup_bv(hipStream_t s, const SetupArgs& a, int nsl, const double2* m, const double2* rinv, double2* bv,
              int nblk, const int* klo, int win, double2* bs);
void setup_rdij(hipStream_t s, const SetupArgs& a, const Band& Wb, const double2* m, const int* g_start, int GL,
                const int* q_start, int QL, double2* rd /* packed, w_elems */);
struct TxDesc {
    int kind, L, K, N, fft, ifb, ts, cp, zg, proto;
    double norm, phase0, rx_scale;
};
// FP64 matrix-core peak microbenchmark: blocks x 4 waves, each `iters` x 8
// independent v_mfma_f64_16x16x4_f64 (2048 flops each)
static constexpr int PEAK_MFMA_PER_ITER = 8;
void launch_mfma_f64_peak(hipStream_t s, int blocks, int iters, double* out);
void setup_tx_matrix(hipStream_t s, const TxDesc& d, const double* proto, double2* G, double2* Q);
// D = Q^H H G of lane `lane` of a Jakes batch `ir` (dsce_transmission_matrix, test probe)
void setup_transmission_matrix(hipStream_t s, const ChannelK& ch, int LK, const double2* ir, int R, int lane,
                               const double2* G, const double2* Q, const int* qlo, const int* qhi, double2* hg,
                               double2* D);
void setup_fused_stage(hipStream_t s, const Band& Wb, int LK, int NP, const double2* w, long long w_elems,
                       const double2* wd, int nslices, const int* pil_blk, const int* pilot_pos, int ncol,
                       double2* wpil, double2* wda);
void setup_wpair(hipStream_t s, const Band& Wb, int NP, const double2* w, long long w_elems, const PairBand& P,
                 double2* wp, long long wp_elems, int nslices, double* w3);
void setup_w_extent(hipStream_t s, const Band& Wb, int NP, const double2* w, long long w_elems, int nslices, int* lohi);
void setup_w(hipStream_t s, const SetupArgs& a, const Band& Wb, long long w_elems, const double2* rd,
             const double2* rinv /* NP x NP */, double2* w /* packed */, double2* wd /* LK x NP */);

}  // namespace dsce
