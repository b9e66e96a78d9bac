/*
 * dsce.h — C-ABI of the MI355X doubly-selective channel-estimation engine
 * (libdsce.so).  Plain C types only: pointers + sizes, no torch/HIP types.
 *
 * Reference: rnissel/Channel-Estimation (MATLAB).  The reference has no native
 * layer; these entry points are what a MEX gateway behind the reference's
 * class surfaces binds (see INTEGRATION.md for the gateway and ctypes stubs):
 *
 *   dsce_set_channel      <- Channel.FastFading(...) ctor        FastFading.m:25-192
 *   dsce_channel_realise  <- FastFading.NewRealization +
 *                            .ImpulseResponse / GetConvolutionMatrix
 *                                                               FastFading.m:194-250, :276-295
 *   dsce_add_scheme       <- the operator set of the script     DoublySelectiveChannelEstimation.m:191-205
 *                            (G_*, Q_*, precoders of
 *                             ImaginaryInterferenceCancellationAtPilotPosition.m:37-229,
 *                             PilotMapping_OFDM script:134-142)
 *   dsce_set_snr          <- M_SNR_dB / Pn_time / NrIterations   script:18, :33, :243, :398
 *   dsce_build_mmse       <- correlation matrices + MMSE W      script:208-313 (+ FastFading.m:321-407);
 *                            the 'MMSE' slot of PilotSymbolAidedChannelEstimation
 *                            (stubbed with error() at PSACE.m:110-111)
 *   dsce_run              <- the Monte-Carlo loop body          script:350-564
 *                            ('MMSE' ChannelInterpolation, PSACE.m:128-129, per stage)
 *   dsce_mmse_onetap      <- PilotSymbolAidedChannelEstimation.ChannelInterpolation,
 *                            method 'MMSE' (PSACE.m:128-129 stub): h_hat = diag(sum_p W_p hP_p),
 *                            script:417-428
 *   dsce_get_correlation / dsce_get_W <- R_hP*, W_MMSE_*          script:210-313 (parity probes)
 *   dsce_tx_matrices      <- OFDM/FBMC.GetTXMatrix / GetRXMatrix OFDM.m:184-218, FBMC.m:318-354
 *   dsce_set_interpolation <- PilotSymbolAidedChannelEstimation.ChannelInterpolation,
 *                            'linear'/'nearest'/'FullAverage'/'MovingBlockAverage'
 *                            (PSACE.m:73-107, :115-133) as its LK x NP weight matrix
 *   dsce_set_noise_slot   <- separate n_FBMC / n_OFDM draws     SimpleVersion_DoublyFlat.m:125-126
 *
 * Conventions
 *  - Return 0 on success, a negative DSCE_E* code on failure; the message is
 *    available from dsce_last_error(ctx).  No C++ exception crosses the ABI.
 *  - Complex numbers are interleaved (re, im) doubles; matrices are
 *    column-major like MATLAB (R2018a+ interleaved complex storage).
 *  - Indices are 0-based (a MEX gateway subtracts 1).
 *  - Host buffers are caller-owned and only read/written during the call;
 *    device memory and the HIP stream are owned by the context.
 *  - One context per thread per GPU; no global mutable state besides the HIP
 *    runtime.  A context binds to one HIP device at dsce_create.
 *
 * Random streams (shared with the CPU oracle, oracle/philox.py).
 *  Philox4x32-10 (Salmon et al. 2011), key = (seed & 0xffffffff, seed >> 32),
 *  counter = (idx, rep & 0xffffffff, rep >> 32, stream << 16 | sub).
 *  u53(a,b) = ((a>>5)*2^26 + (b>>6)) * 2^-53.
 *    THETA  (1, 0)   Doppler angles, element e = tap + Ntap*path (MATLAB
 *                    rand([Ntap 1 Paths]) column-major, FastFading.m:227):
 *                    counter e/2, words (0,1) for even e, (2,3) for odd e.
 *    PHI    (2, 0)   random phases, same layout (FastFading.m:233).
 *    BITS   (3, s)   data bits of scheme slot s (script:355-357): bit i is bit
 *                    (i & 31) of word ((i>>5) & 3) of counter i>>7.
 *    PILOTS (4, s)   pilot symbol indices (script:365-367): pilot j is word
 *                    (j & 3) of counter j>>2, masked to log2(M) bits.
 *    NOISE  (5, k + 256 g)  AWGN of SNR index k, shared by all schemes of
 *                    noise slot g (default 0: all schemes, script:399):
 *                    sample e: normal pair of counter e, where a normal pair is
 *                    u1=u53(w0,w1), u2=u53(w2,w3);
 *                    re = sqrt(-2 log(1-u1)) cos(2 pi u2), im = ... sin(2 pi u2).
 *    THETA  (1, 0)   max_doppler == 0: tap q (q-th non-zero tap) is
 *                    1/sqrt(2) sqrt(PDPn) (re + j im) of the normal pair of
 *                    counter q (FastFading.m:244).
 *    THETA  (1, 1)   discrete Doppler models: Doppler bin f = -nd..nd of tap q is
 *                    the normal pair of counter (f + nd) + (2 nd + 1) q
 *                    (GaussUncorr1 / GaussUncorr2, FastFading.m:207-211).
 *
 * Error counters (dsce_run): int64 array of shape
 *   [n_schemes][2 csi: 0 = MMSE estimate, 1 = perfect CSI][2 edge: 0 = all bits,
 *    1 = no-edge bits][n_snr][1 + n_iter stages: 0 = one-tap, i = IC iteration i]
 * (C order, last index fastest).  BER = count / bits, bits from dsce_bits_per_rep.
 */
#ifndef DSCE_H
#define DSCE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSCE_ABI_VERSION 7

#define DSCE_OK 0
#define DSCE_EINVAL -1      /* bad argument / shape */
#define DSCE_EHIP -2        /* HIP runtime error */
#define DSCE_ESTATE -3      /* call order (e.g. run before build_mmse) */
#define DSCE_ENOMEM -4

/* How dsce_run sums the members of a context (dsce_group_info) */
#define DSCE_REDUCE_NONE 0  /* a single-device context (dsce_create)                       */
#define DSCE_REDUCE_RCCL 1  /* ncclAllReduce (sum) of the members' device counters, RCCL    */
                            /* over xGMI: dsce_create_multi with distinct devices           */
#define DSCE_REDUCE_HOST 2  /* a device repeats in dsce_create_multi's list (one RCCL rank  */
                            /* per device): the members' counters are summed on the host    */

typedef struct dsce_ctx dsce_ctx;

typedef struct {
    int32_t n_samples;          /* N                                          */
    int32_t n_taps;             /* length of the sampled PDP (incl. zero taps) */
    double sampling_rate;       /* Hz                                         */
    double max_doppler;         /* Hz (FastFading.m:42); 0 = time-invariant    */
                                /* block fading (FastFading.m:241-246)         */
    int32_t n_paths;            /* sum-of-sinusoids paths (FastFading.m:179)   */
    int32_t doppler_model;      /* 0 = 'Jakes', 1 = 'Uniform' (sum of sinusoids, */
                                /* FastFading.m:222-238), 2 = 'Discrete-Jakes', */
                                /* 3 = 'Discrete-Uniform' (IFFT of the discrete */
                                /* Doppler spectrum, FastFading.m:158-177,      */
                                /* :203-221; fD/df <= 0.5 sets fD = 0, :153-156) */
    const double* pdp_norm;     /* n_taps, PowerDelayProfileNormalized (:129) */
} dsce_channel_desc;

typedef struct {
    int32_t n_subcarriers;      /* L                                          */
    int32_t n_symbols;          /* K; LK = L*K columns of G and Q              */
    int32_t n_tx_symbols;       /* columns of P: NP + ND                       */
    int32_t n_pilots;           /* NP                                          */
    int32_t n_data;             /* ND                                          */
    int32_t mod_order;          /* M (power of two)                            */
    int32_t bits_per_symbol;    /* log2(M)                                     */
    int32_t despread;           /* 1: x_hat = P^H (y./h), data = entries NP..  (script:436) */
    int32_t real_detect;        /* 1: real() before detection (FBMC-OQAM)      */
    int32_t bits_slot;          /* RNG sub-stream for the data bits            */
    int32_t pilot_slot;         /* RNG sub-stream for the pilots               */
    double kappa;               /* pilot scaling, script:140-142               */
    double data_div;            /* divisor before detection, script:430/437/444 */
    const double* G;            /* N x LK complex, s = G x                     */
    const double* Q;            /* N x LK complex, y = Q^H r                   */
    const double* P;            /* LK x n_tx_symbols complex, x = P [xP; xD]   */
    const int32_t* pilot_pos;   /* n_pilots positions in 0..LK-1               */
    const int32_t* data_pos;    /* n_data positions (select mode)              */
    const uint8_t* considered;  /* n_data no-edge flags (script:151-172)       */
    const double* symbols;      /* M complex, SymbolMapping sorted by bit label */
} dsce_scheme_desc;

/* On-GPU producer of the transmit / receive matrices,
 * replacing Modulation.OFDM/FBMC.GetTXMatrix / GetRXMatrix (OFDM.m:184-218,
 * FBMC.m:318-354): column l + L k of G is the modulated unit impulse of
 * subcarrier l, symbol k, evaluated in closed form per element instead of L
 * Modulation() calls; Q = GetRXMatrix' = G * rx_scale with the OFDM cyclic-
 * prefix samples zeroed (OFDM.m:216-217). */
typedef struct {
    int32_t kind;               /* 0 = OFDM, 1 = FBMC Hermite-OQAM             */
    int32_t n_subcarriers;      /* L                                          */
    int32_t n_symbols;          /* K                                          */
    int32_t n_samples;          /* N = Nr.SamplesTotal                         */
    int32_t fft_size;           /* Implementation.FFTSize                      */
    int32_t intermediate_bin;   /* Implementation.IntermediateFrequency       */
    int32_t time_spacing;       /* Implementation.TimeSpacing (samples)        */
    int32_t cyclic_prefix;      /* OFDM Implementation.CyclicPrefix            */
    int32_t zero_guard;         /* OFDM Implementation.ZeroGuardSamples        */
    int32_t proto_len;          /* FBMC Nr.SamplesPrototypeFilter              */
    double norm;                /* Implementation.NormalizationFactor          */
    double initial_phase;       /* FBMC Implementation.InitialPhaseShift       */
    double rx_scale;            /* GetRXMatrix scale (OFDM L F/SR, FBMC L/(SR T)) */
    const double* prototype;    /* FBMC PrototypeFilter.TimeDomain (proto_len) */
} dsce_tx_desc;

/* Dimensions of a configured scheme, so a binding sizes every output from the
 * engine's own state (dsce_scheme_dims).  n_counters = length of dsce_run's
 * err_counts (all schemes). */
typedef struct {
    int32_t n_samples;          /* N                                          */
    int32_t n_taps;             /* length of the sampled PDP (ImpulseResponse columns) */
    int32_t lk;                 /* L * K                                      */
    int32_t n_pilots;           /* NP                                         */
    int32_t n_data;             /* ND                                         */
    int32_t n_tx_symbols;       /* NP + ND                                    */
    int32_t n_schemes;
    int32_t n_snr;
    int32_t n_iter;
    int64_t n_counters;
} dsce_dims;

/* Per-stage trace of one unit (dsce_trace_unit_ex).  Every pointer is optional
 * (null: not returned).  Complex buffers interleaved; "stage" s = 0 one-tap,
 * s = i IC iteration i; (1 + n_iter) rows, each LK (or NP / ND) long.
 * Entries no kernel of the path forms are NaN (since ABI 4; ABI 3 left 0):
 * e.g. the pilot rows of yperf_stages on the fused perfect-CSI paths, and
 * hest_stages / yest_stages rows of symbols a stage kernel does not visit. */
typedef struct {
    double* y;                  /* LK: y = Q'r                                    script:406-409 */
    double* h_perfect;          /* LK: diag(D), D = Q'HG                           script:388-393 */
    double* hp_stages;          /* (1+n_iter) x NP: LS pilot estimates             script:412-414, :487-489 */
    double* hest_stages;        /* (1+n_iter) x LK: diag(D_hat)                    script:417-428, :493-515 */
    double* yest_stages;        /* (1+n_iter) x LK: y_est = y - (D_hat - diag) v   script:482-484 (row 0 = y) */
    double* yperf_stages;       /* (1+n_iter) x LK: y_perf = y - (D - diag h) u    script:541-543 (row 0 = y;
                                   data rows only on the fused perfect-CSI paths) */
    int32_t* dec_est;           /* (1+n_iter) x ND: detected symbol index, MMSE    script:431, :527 */
    int32_t* dec_perf;          /* (1+n_iter) x ND: detected symbol index, perfect script:453, :548 */
} dsce_trace;

/* Kernel paths (dsce_path_info) */
#define DSCE_PATH_WPAIR3_FUSED    (1u << 0)   /* k_pilot_pre + k_wpair3 with the MMSE stage in its epilogue */
#define DSCE_PATH_WPAIR3          (1u << 1)   /* k_wpair3: MFMA pair-tile contraction, 3M products        */
#define DSCE_PATH_WPAIR4M         (1u << 2)   /* retired in r03 (k_wpair, 4M products); never set          */
#define DSCE_PATH_WCONTRACT_VALU  (1u << 3)   /* k_wcontract_valu                                         */
#define DSCE_PATH_PIC_MFMA        (1u << 4)   /* retired in ABI 4 (k_pic_mfma); never set                  */
#define DSCE_PATH_PIC_CHAIN       (1u << 5)   /* retired in ABI 4 (k_pic_chain); never set                 */
#define DSCE_PATH_PIC_PASSES      (1u << 6)   /* perfect-CSI IC as two banded passes per iteration         */
#define DSCE_PATH_STAGE_FUSED     (1u << 7)   /* k_ls + k_stage_fused                                      */
#define DSCE_PATH_STAGE_SPLIT     (1u << 8)   /* k_ls_hest + k_detect + k_precode                          */
#define DSCE_PATH_NOISE_FUSED     (1u << 9)   /* AWGN drawn inside the Q^H pass                            */
#define DSCE_PATH_PIC_FFT         (1u << 10)  /* k_pic_fft: perfect-CSI IC chain by FFT (OFDM, VALU)       */
#define DSCE_PATH_MIC_FFT         (1u << 11)  /* MMSE IC as Q' H_hat G by FFT (OFDM; with DSCE_PATH_MIC_STAGES) */
#define DSCE_PATH_TXRX_FFT        (1u << 12)  /* k_txrx_fft: TX + channel + noisy receiver front by FFT (OFDM) */
#define DSCE_PATH_PILOT_FUSED     (1u << 13)  /* retired in r03 (k_mic_fft's fused pilot pass); never set     */
#define DSCE_PATH_MIC_STAGES      (1u << 14)  /* k_mic_pilot + k_mic_data: every MMSE stage of an FFT-form OFDM
                                                 scheme in one launch pair; k_pic_fft with the perfect-CSI stage 0 */
#define DSCE_PATH_MIC_LR          (1u << 15)  /* ... with the low-rank tap operator: taps = T_k Z, Z = Bz hP once per
                                                 unit and stage (dsce_structured_check out[5]) */
#define DSCE_PATH_PIC_POLY        (1u << 16)  /* perfect-CSI IC of a polyphase scheme (FBMC; OFDM with L = 48) as
                                                 IDFT-L per symbol + window sums per residue + DFT-L per symbol
                                                 (k_poly_syn / k_poly_chan / k_poly_ana, option pic_poly) */
#define DSCE_PATH_WROW3           (1u << 17)  /* unfused W contraction of 32-row blocks as one GEMM per row tile,
                                                 B = hP v_c (k_wrow3, option wrow) */

int dsce_abi_version(void);
int dsce_device_count(int* count);

int dsce_create(int hip_device, dsce_ctx** out);
/* Frees the context (every buffer, event and the stream) and returns DSCE_OK,
 * or DSCE_EHIP if a HIP call of the teardown failed (the context is freed
 * either way; the first failing call is named on stderr).  ABI 6: returned
 * void up to ABI 5 (a double free went unseen). */
int dsce_destroy(dsce_ctx* ctx);
const char* dsce_last_error(const dsce_ctx* ctx);

/* Multi-device context (ABI 7; SURVEY §8e, north_star: "realisations shard
 * embarrassingly across the 8 GPUs of one node with a single RCCL all-reduce"),
 * so a host that stays one MATLAB process (README.md:19-20; the loop of
 * DoublySelectiveChannelEstimation.m:350-564) drives every GPU through one
 * handle.  Member i is a context on devices[i] (member 0 is the returned
 * handle).
 *  - Every configuration call — dsce_set_channel, dsce_set_snr,
 *    dsce_add_scheme, dsce_build_mmse (members in parallel: setup is
 *    replicated per device), dsce_set_batch, dsce_set_noise_slot,
 *    dsce_set_interpolation, dsce_set_option, dsce_enable_mse,
 *    dsce_enable_timing — applies to every member (member 0 first; a member's
 *    failure is reported through the handle's dsce_last_error).
 *  - dsce_run splits [first_rep, first_rep + n_rep) into n_devices contiguous
 *    slices on multiples of 64 realisations (dsce/parallel.py shard_range), runs
 *    member i's slice on its own host thread, then sums the members' int64
 *    counters (and MSE sums) with ONE ncclAllReduce per buffer over
 *    communicators from ncclCommInitAll (DSCE_REDUCE_RCCL; devices distinct,
 *    n_devices = 1 included) or on the host when a device repeats
 *    (DSCE_REDUCE_HOST), and adds the total into err_counts once.  The Philox
 *    streams are keyed by the global realisation index, so the counts equal a
 *    single context's bit for bit for any member count.
 *  - Every other call (probes, queries, dsce_kernel_time: member 0's own
 *    launches, i.e. its slice) uses member 0.
 * dsce_destroy on the handle frees every member and communicator. */
int dsce_create_multi(const int32_t* devices, int32_t n_devices, dsce_ctx** out);
/* Members of a context: *n_devices, their HIP devices (optional, n_devices
 * entries) and *reduce = DSCE_REDUCE_* (each pointer optional). */
int dsce_group_info(dsce_ctx* ctx, int32_t* n_devices, int32_t* devices, int32_t* reduce);

int dsce_set_channel(dsce_ctx* ctx, const dsce_channel_desc* desc);
int dsce_set_snr(dsce_ctx* ctx, const double* pn_time, int32_t n_snr, int32_t n_iter);
int dsce_add_scheme(dsce_ctx* ctx, const dsce_scheme_desc* desc, int32_t* scheme_id);

/* Builds R_hP, R_hP,est, R_hP,est(no interference), R_Dij,hP and the two MMSE
 * estimators W / W0 for every SNR on the GPU, zeroing |.| < zero_threshold
 * like script:263-264, :287-289, :306-308. */
int dsce_build_mmse(dsce_ctx* ctx, double zero_threshold);

/* Repetitions per device batch (default 8192); larger batches fill the GPU
 * better at the cost of HBM for per-unit state. */
int dsce_set_batch(dsce_ctx* ctx, int32_t reps_per_batch);

/* Runs realisations [first_rep, first_rep + n_rep) for every scheme and SNR and
 * ADDS the bit-error counts into err_counts (layout above).  Synchronous.  Any
 * n_rep >= 0 (the script's NrRepetitions = 25 / 1000, script:19 / :44): the
 * device works in whole wavefronts of 64 realisations, and the padding
 * realisations of a tail wave are simulated but counted nowhere (nor in the MSE
 * sums), so counts over [a, b) equal the sum over any split of [a, b). */
int dsce_run(dsce_ctx* ctx, uint64_t seed, uint64_t first_rep, uint64_t n_rep, int64_t* err_counts);

/* Bits per realisation of a scheme: [0] all data bits, [1] no-edge bits. */
int dsce_bits_per_rep(dsce_ctx* ctx, int32_t scheme_id, int64_t* bits2);

/* MMSE one-tap channel for n_units LS pilot-estimate vectors (the 'MMSE' slot of
 * PilotSymbolAidedChannelEstimation): hp_ls is NP x n_units complex
 * (column-major), h_out LK x n_units complex; variant 0 = W, 1 = W0. */
int dsce_mmse_onetap(dsce_ctx* ctx, int32_t scheme_id, int32_t snr_index, int32_t variant, const double* hp_ls,
                     int32_t n_units, double* h_out);

/* G (and Q, each optional) as N x LK complex column-major host buffers. */
int dsce_tx_matrices(dsce_ctx* ctx, const dsce_tx_desc* desc, double* G_out, double* Q_out);

/* Noise slot of a scheme (0..255, default 0): schemes of one slot share the AWGN
 * draw of an SNR point (script:399-403); SimpleVersion_DoublyFlat.m:125-126
 * draws n_FBMC and n_OFDM separately (two slots). */
int dsce_set_noise_slot(dsce_ctx* ctx, int32_t scheme_id, int32_t slot);

/* One-tap channel estimate by a fixed linear interpolation of the LS pilot
 * estimates, h_hat = I hP, instead of the MMSE estimator: the non-'MMSE'
 * methods of PilotSymbolAidedChannelEstimation.ChannelInterpolation
 * (PSACE.m:115-133: 'linear' / 'nearest' scatteredInterpolant weights,
 * 'FullAverage', 'MovingBlockAverage' — all linear in the LS values).
 * I is LK x NP complex, column-major.  The scheme then needs no
 * dsce_build_mmse, and dsce_run requires n_iter == 0 (no W for the IC
 * iterations).  Used by the doubly-flat script, SimpleVersion_DoublyFlat.m:143-145. */
int dsce_set_interpolation(dsce_ctx* ctx, int32_t scheme_id, const double* interp);

/* ---- parity probes (same kernels as dsce_run) ---------------------------- */
/* ImpulseResponse of realisation `rep`: N x n_taps complex, column-major. */
int dsce_channel_realise(dsce_ctx* ctx, uint64_t seed, uint64_t rep, double* ir_out);
/* D = Q^H H G of realisation `rep` for a scheme (script:381-393, the matrix whose
 * diagonal is the perfect-CSI one-tap channel h and whose off-diagonal part the
 * perfect-CSI IC subtracts, script:541-543): LK x LK complex, column-major.  The
 * Monte-Carlo kernels never form D; this probe builds it
 * from the context's dense G / Q and the run's Jakes realisation (ABI 7). */
int dsce_transmission_matrix(dsce_ctx* ctx, int32_t scheme_id, uint64_t seed, uint64_t rep, double* d_out);
/* R_hP (NP x NP), R_est / R_noI (n_snr x NP x NP, each NP x NP column-major). */
int dsce_get_correlation(dsce_ctx* ctx, int32_t scheme_id, double* r_hp, double* r_est, double* r_noi);
/* W (variant 0) or W0 (variant 1) of SNR index k in the reference layout:
 * vector of LK*LK*NP complex, index r + LK*c + LK*LK*p (script:283). */
int dsce_get_W(dsce_ctx* ctx, int32_t scheme_id, int32_t snr_index, int32_t variant, double* w_out);
/* Per-unit trace of one (rep, snr): y (LK), then for stages 0..n_iter the LS
 * pilot estimates (NP each) and the MMSE one-tap channel diag(D_hat) (LK each),
 * and the perfect-CSI diag(D) (LK).  Buffers complex, sized by the caller. */
int dsce_trace_unit(dsce_ctx* ctx, int32_t scheme_id, uint64_t seed, uint64_t rep, int32_t snr_index,
                    double* y, double* hp_stages, double* hest_stages, double* h_perfect);

/* Channel-estimation MSE (build-defined: the reference computes no MSE, so
 * this output is parity-unpinned against MATLAB and checked against the
 * oracle only).  While enabled, every dsce_run adds, per scheme, SNR point and
 * stage (0 = one-tap, i = IC iteration i), the sum over realisations and the
 * LK positions of |h_hat - h|^2, h_hat = diag(D_hat) the stage's MMSE (or
 * interpolation) estimate and h = diag(D) the perfect-CSI one-tap channel of
 * script:450-466; and per scheme and SNR point the sum of |h|^2 (NMSE =
 * err / pow).  err_sum [n_schemes][n_snr][1 + n_iter], pow_sum
 * [n_schemes][n_snr], totals since the last dsce_enable_mse(ctx, 1). */
int dsce_enable_mse(dsce_ctx* ctx, int32_t enable);
int dsce_get_mse(dsce_ctx* ctx, double* err_sum, double* pow_sum);

/* Same kernels as dsce_run (a 64-realisation batch starting at `rep`, the traced
 * unit at its lane 0), with every stage's intermediate quantities of one
 * (rep, snr) unit returned through `out` (see dsce_trace). */
int dsce_trace_unit_ex(dsce_ctx* ctx, int32_t scheme_id, uint64_t seed, uint64_t rep, int32_t snr_index,
                       const dsce_trace* out);

/* ---- engine state ------------------------------------------------------- */
int dsce_scheme_dims(dsce_ctx* ctx, int32_t scheme_id, dsce_dims* dims);
/* Which kernels a scheme's last dsce_run / trace used: DSCE_PATH_* bits. */
int dsce_path_info(dsce_ctx* ctx, int32_t scheme_id, uint32_t* flags);
/* Kernel-selection options (defaults = the measured-best path; each other value
 * selects a real fallback, reached by the parity tests):
 *   xcd (XCD-aware work order), fuse_stage (MMSE stage in the contraction's
 *   epilogue), pic_chain (3: perfect-CSI IC chain by FFT where the scheme's G / Q
 *   allow it, 0: two banded passes per iteration), pfuse, stage_split, stage_rb
 *   (4|8|16), noise_fuse, snr_chunk (0 all), jakes_rpw (1|2), wtrim (read by
 *   dsce_build_mmse), wcontract_valu (the VALU contraction, also the fallback
 *   without pair tiles), mmse_ic (1: the MMSE branch of an FFT-form OFDM scheme
 *   as y - Q'(H_hat (G v)) + diag(D_hat) v with H_hat = E{H | hP}, every stage in
 *   k_mic_pilot + k_mic_data and the perfect-CSI stage 0 in k_pic_fft; equal to
 *   the W contraction of script:482-511 to rounding, checked at dsce_build_mmse;
 *   0: the W contraction everywhere), jakes_win, txrx_fft, jakes_mom (the Jakes
 *   taps of the read windows: 2 = Taylor anchors over runs of windows, 1 = one
 *   anchor per window, 0 = the recurrence; each only where its truncation stays
 *   below rounding), realise_win (1: dsce_channel_realise forms only the samples
 *   the schemes' windows read, zero elsewhere, with the run's Jakes kernels),
 *   tx_rows (1: TX symbols of a row-local precoder drawn row-parallel), snr_base
 *   (0..255: the noise of SNR index k is sub-stream snr_base + k, so a rank
 *   serving SNR points [b, ...) of a sweep draws the one-rank run's noise),
 *   mic_lr (1: the MMSE IC's estimated taps in the low-rank form T_k Z where the
 *   fit reproduces Bv to rounding, dsce_structured_check; 0: the tap GEMM Bv hP),
 *   pic_poly (1: the perfect-CSI IC passes of a scheme whose G and Q factorise as real windows x
 *   subcarrier tones, G[n, l + L k] = A_k[n] e^(2 pi i l n / L) C[l][k], checked
 *   entry by entry to 1e-12 at dsce_add_scheme, with L = 24 or 48, as an IDFT-L
 *   per symbol, window sums per residue n mod L around the channel, and a DFT-L
 *   per symbol, DSCE_PATH_PIC_POLY, the default; 0: the two banded passes),
 *   wrow (1: the unfused W contraction of 32-row blocks — FBMC, C5 — as one
 *   GEMM per 16-row tile over (column, pilot) with B = hP v_c, no per-tile
 *   epilogue, DSCE_PATH_WROW3; 0: k_wpair3's pair tiles), jakes_grp2 (1, the
 *   default: a channel with two non-zero taps forms the Jakes taps of the read
 *   windows with k_jakes_grp2 — both taps per wave, each Philox block drawn
 *   once; 0: k_jakes_grp, one tap per block; r06).
 * Retired in r06 (measured neutral in r04 / r05; DSCE_EINVAL): pic_skip (the
 * perfect-CSI fixed-point exit), ic_streams (the chain on a second stream /
 * beside the pilot pass in one launch, k_ic_pair).
 * Retired in r03 (the r01-r02 variants they selected are gone; DSCE_EINVAL):
 * wpair_3m, wda_3m, streams, qidx, stage0_fft, mic_mfma, pilot_fft, mic_yic,
 * pilot_fuse, mic2.  Unknown names return DSCE_EINVAL. */
int dsce_set_option(dsce_ctx* ctx, const char* name, int64_t value);
int dsce_get_option(dsce_ctx* ctx, const char* name, int64_t* value);

/* ---- measurement -------------------------------------------------------- */
/* When enabled, dsce_run records HIP events around every launch of each kernel
 * on the stream it runs on; dsce_kernel_time returns (launches, total ms).
 * "ic_stages" is the span of the FFT-form OFDM IC group (k_pic_fft,
 * k_mic_pilot, k_mic_data, in sequence on the context's stream). */
int dsce_enable_timing(dsce_ctx* ctx, int32_t enable);
int dsce_kernel_time(dsce_ctx* ctx, const char* kernel, int64_t* launches, double* total_ms);
/* Algorithmic work of one realisation of a scheme (support-aware): complex
 * multiply-accumulates of the MMSE contraction kernel over W's off-diagonal
 * (row, column) pairs (including, when the last dsce_run fused the MMSE stage
 * into it, the diag(D_hat) = Wd hP products) and the number of W bytes streamed
 * per contraction launch. */
int dsce_work_model(dsce_ctx* ctx, int32_t scheme_id, double* wcontract_cmac_per_rep, double* w_bytes_per_snr);
/* Algorithmic work per realisation of one timed kernel group (the names of
 * dsce_kernel_time) as configured by the last dsce_run, summed over the
 * schemes that ran it: flops (8 per complex multiply-accumulate, 5 n log2 n per
 * n-point DFT; transcendentals and RNG integer work not counted) and the
 * compulsory HBM bytes (each operand read once per realisation / unit, each
 * result written once).  Modelled: the FFT-form OFDM chain (k_jakes, tx,
 * rx_front, perfect_ic, k_mic_pilot, k_mic_data, and ic_stages = the sum of the
 * last three), the polyphase perfect-CSI
 * passes (perfect_ic of FBMC / L = 48 OFDM) and the W contraction (k_wcontract);
 * 0 = not modelled for the path that ran.  DESIGN.md section 4
 * lists the per-unit formulas. */
int dsce_kernel_work(dsce_ctx* ctx, const char* kernel, double* flops_per_rep, double* bytes_per_rep);
/* The guard of the structured MMSE IC (D_hat = Q' H_hat G, DSCE_PATH_MIC_FFT),
 * evaluated at dsce_build_mmse: out[0] = worst over the (variant, SNR) slices of
 * max |Q' H_hat G - W_thr| / (rtol max |W|) over every entry the IC uses, with
 * the slice's rounding bar rtol = min(1e-9, max(1e-11, 4e-16 ||R||_1
 * ||pinv(R)||_1)) (the path is kept iff <= 1), out[1] = the largest absolute
 * deviation, out[2] = the largest |W|, out[3] = the largest rtol of the slices.
 * out[0..2] = -1 when the scheme is not eligible (the W contraction runs).
 * The low-rank form of its tap operator (Bv = T Bz, T_k the J0 kernel summed
 * over pilot symbol k's window; option mic_lr): out[4] = max |Bv - T Bz| /
 * max |Bv| of the fit (-1: not attempted), out[5] = 1 if the operator was
 * built and kept (eligible), else 0 — a run uses it only with the options
 * mic_lr = 1 and mic_net bit 0 set, which DSCE_PATH_MIC_LR of dsce_path_info
 * reports after the run — out[6] = the worst slice's deviation over its rounding
 * bar min(1e-9, max(1e-13, 4e-16 ||R||_1 ||pinv(R)||_1)) max |Bv| (the operator
 * is kept iff <= 1). */
int dsce_structured_check(dsce_ctx* ctx, int32_t scheme_id, double* out7);
/* Measured FP64 matrix-core peak of the context's GPU: back-to-back
 * v_mfma_f64_16x16x4_f64 on independent accumulators, 8 waves per SIMD,
 * best of 3 timed launches (TFLOP/s). */
int dsce_fp64_mfma_peak(dsce_ctx* ctx, double* tflops);

#ifdef __cplusplus
}
#endif

#endif /* DSCE_H */
