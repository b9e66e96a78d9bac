// dsce_api.hip — C-ABI (include/dsce.h) and host-side orchestration of the
// HIP engine: operator packing (banded / CSR / compact layouts), device memory,
// the setup pipeline (script:208-313) and the batched Monte-Carlo loop
// (script:350-564).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <cstdio>
#include <thread>
#include <vector>

#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include "dsce.h"
#include "dsce_kernels.h"

// roctx ranges around the run, each device batch, the counter all-reduce and
// the setup entry points (tracing): named spans on the host
// timeline under `rocprofv3 --marker-trace`, no-ops without a profiler
struct TraceRange {
    explicit TraceRange(const char* m) { roctxRangePushA(m); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

namespace dsce {

struct HipError : std::runtime_error {
    HipError(hipError_t e, const char* what, const char* file, int line)
        : std::runtime_error(std::string("HIP error '") + hipGetErrorString(e) + "' at " + file + ":" +
                             std::to_string(line) + " (" + what + ")") {}
};
struct ApiError : std::runtime_error {
    int code;
    ApiError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

static inline double2 cx(const double* p, size_t i) { return make_double2(p[2 * i], p[2 * i + 1]); }
static inline bool nz(double2 v) { return v.x != 0.0 || v.y != 0.0; }

struct HostBand {
    int rb = DSCE_RB;
    std::vector<int> row0, nrows, klo, khi;
    std::vector<long long> off;
    std::vector<double2> vals;
    long long elems = 0;
};

// rows [0, nrow) grouped in blocks of at most rb rows; range(row) -> [lo, hi).
// split_disjoint: a block also ends where the next row's range does not overlap
// the block's union (block-diagonal operators such as the OFDM estimator).
template <class RangeFn>
static HostBand band_geometry(int nrow, RangeFn range, int kscale, int rb = DSCE_RB, bool split_disjoint = false) {
    HostBand b;
    b.rb = rb;
    long long off = 0;
    int r0 = 0;
    while (r0 < nrow) {
        int lo = 1 << 30, hi = -1, nr = 0;
        for (int r = r0; r < nrow && nr < rb; ++r) {
            int a, c;
            range(r, a, c);
            if (split_disjoint && nr > 0 && c > a && hi >= 0 && (a >= hi || c <= lo)) break;
            if (c > a) {
                lo = std::min(lo, a);
                hi = std::max(hi, c);
            }
            ++nr;
        }
        if (hi < 0) { lo = 0; hi = 0; }
        b.row0.push_back(r0);
        b.nrows.push_back(nr);
        b.klo.push_back(lo * kscale);
        b.khi.push_back(hi * kscale);
        b.off.push_back(off);
        off += (long long)(hi - lo) * kscale * rb;
        r0 += nr;
    }
    b.elems = off;
    return b;
}

// CMACs of one contraction over a packed W band (rows x (column, pilot) entries)
// and how many of them are (r, r) pairs, which the band stores as zeros.
static void band_work(const HostBand& b, int NP, long long& total, long long& diag) {
    total = diag = 0;
    for (size_t blk = 0; blk < b.row0.size(); ++blk) {
        const int clo = b.klo[blk] / NP, chi = b.khi[blk] / NP;
        total += (long long)b.nrows[blk] * (b.khi[blk] - b.klo[blk]);
        for (int r = b.row0[blk]; r < b.row0[blk] + b.nrows[blk]; ++r)
            if (r >= clo && r < chi) diag += NP;
    }
}

struct Scheme {
    dsce_scheme_desc d{};
    int N = 0, LK = 0;
    std::vector<double2> G, Q, P;   // dense host copies (column-major)
    std::vector<int> pilot_pos, data_pos;
    std::vector<uint8_t> considered;
    std::vector<double2> symbols;
    SchemeK k{};
    HostBand gband, qband, hband, wband, wband_struct;   // wband: trimmed after build_mmse
    Band Wb{};
    long long w_elems = 0, w_struct = 0;
    double2* W = nullptr;
    double2* Wd = nullptr;
    double* Wp3 = nullptr;          // pair-tile copy of W as Re / Im / Re+Im planes (k_wpair3; null: not eligible)
    double2* Wpil = nullptr;        // fused MMSE stage operands (null: not eligible)
    double2* WdA = nullptr;
    int* pil_c0 = nullptr;
    double2* Bv = nullptr;          // structured MMSE IC operator (k_mic_pilot / k_mic_data; null: not eligible)
    double2* Bs = nullptr;
    int* pblk = nullptr;            // QH blocks with pilot rows (k_mic_pilot)
    int* pmask = nullptr;           // [QH blk] 1 = holds pilot rows
    int npb = 0;
    int* dblk = nullptr;            // QH blocks without pilot rows (k_mic_data)
    int ndb = 0;
    // low-rank form of Bv (build_mic_lr): Bv[q][n][p] = sum_k T_k[n] Bz[q k][p]; null: not eligible
    double2* Bz = nullptr;          // [var][snr][ntap * MIC_NB][NP]
    double* Tw = nullptr;           // [QH blk][MIC_NB][24]
    double* Ts = nullptr;           // [QH blk][MIC_NB]
    double lr_resid = -1.0;         // max |Bv - T Bz| / max |Bv| of the fit (-1: not built)
    double lr_ratio = -1.0;         // worst slice's deviation / its rounding bar (<= 1: kept)
    long long wp_elems = 0, wp_exec = 0;
    long long w_diag = 0;           // (r, r) pairs inside the band (stored as zeros: diag(D_hat) comes from Wd)
    unsigned path = 0;              // PATH_* bits of the last dsce_run / trace (dsce_path_info)
    PairBand Pb{};
    std::vector<double2> R_hP, R_est, R_noI;
    bool mmse_ready = false;
    // one-tap estimator given as an interpolation matrix (dsce_set_interpolation,
    // PSACE.m:115-133) instead of the MMSE W: LK x NP, row-major [c][p] like Wd
    bool interp = false;
    std::vector<double2> interp_I;
    int64_t bits_all = 0, bits_noedge = 0;
    std::vector<int> g_start, q_start;
    int GL = 0, QL = 0;
    int maxdelay = 0;
    // build_mic's guard (dsce_structured_check): worst over the (variant, SNR)
    // slices of max |Q' H_hat G - W_thresholded| / (MIC_RTOL max |W|), the largest
    // absolute deviation and the largest |W|; -1 = not evaluated
    double mic_check = -1.0, mic_dev = -1.0, mic_wmax = -1.0;
    double mic_rtol = -1.0;         // the largest per-slice bar max(MIC_RTOL, LR_EPS kappa(R)) used
    // build_poly: largest |G - A w C| / max|G| or the same of Q (-1: not evaluated)
    double poly_resid = -1.0;
    double poly_nnz_a = 0.0, poly_nnz_b = 0.0;   // non-zero window samples of G's / Q's symbols
};

}  // namespace dsce

using namespace dsce;

struct dsce_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    bool chan_set = false;
    ChannelK ch{};
    std::vector<double> pdp_norm;
    std::vector<double> pn;
    int nsnr = 0, niter = 4;
    double* d_pn = nullptr;
    std::vector<std::unique_ptr<Scheme>> schemes;
    int batch = 8192;
    Opts op{};                            // kernel selection (dsce_set_option)
    JakesChunks jk{};                     // samples of the IR a batch needs (update_jakes_chunks)
    int jakes_kind = 0;                   // which Jakes kernel the last batch ran (JAKES_KIND_*)
    size_t jk_nsch = (size_t)-1;          // scheme count jk was computed for
    McBuffers buf{};
    size_t buf_key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<void*> buf_allocs;
    unsigned long long* d_counters = nullptr;
    size_t counters_n = 0;
    // pinned host copy of the counters (r06: the per-run copy back is a direct
    // DMA instead of a staged pageable copy)
    unsigned long long* h_counters = nullptr;
    size_t h_counters_n = 0;
    // channel-estimation MSE (dsce_enable_mse): device sums of the current
    // dsce_run, host totals since the last enable
    bool mse = false;
    double* d_mse = nullptr;                 // [err: ns * nsnr * nstage][pow: ns * nsnr]
    size_t mse_n = 0;
    std::vector<double> mse_host;
    std::vector<void*> allocs;
    bool timing = false;
    std::map<std::string, std::pair<int64_t, double>> ktime;
    struct Ev {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Ev> pending;
    std::vector<hipEvent_t> event_pool;
    // multi-device context (dsce_create_multi, ABI 7): this context is member 0,
    // peers are members 1.. (one context each, configured identically); comms:
    // one RCCL communicator per member (ncclCommInitAll) when the devices are
    // distinct; reduce: DSCE_REDUCE_* (how dsce_run sums the members' counters)
    std::vector<dsce_ctx*> peers;
    std::vector<ncclComm_t> comms;
    int reduce = DSCE_REDUCE_NONE;
};

namespace {

template <class T>
T* dalloc(dsce_ctx* c, size_t n, std::vector<void*>* list = nullptr) {
    void* p = nullptr;
    if (n == 0) n = 1;
    DSCE_HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
    (list ? list : &c->allocs)->push_back(p);
    return (T*)p;
}
template <class T>
T* dupload(dsce_ctx* c, const std::vector<T>& v) {
    T* p = dalloc<T>(c, v.size());
    if (!v.empty()) DSCE_HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

void free_alloc(dsce_ctx* c, void* p) {
    for (auto it = c->allocs.begin(); it != c->allocs.end(); ++it)
        if (*it == p) {
            DSCE_HIP_CHECK(hipFree(*it));
            c->allocs.erase(it);
            return;
        }
}

hipEvent_t get_event(dsce_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    DSCE_HIP_CHECK(hipEventCreate(&e));
    return e;
}

struct Timed {
    dsce_ctx* c;
    dsce_ctx::Ev ev;
    bool on;
    hipStream_t st;
    Timed(dsce_ctx* ctx, const char* name, hipStream_t on_stream = nullptr)
        : c(ctx), on(ctx->timing), st(on_stream ? on_stream : ctx->stream) {
        if (on) {
            ev.name = name;
            ev.a = get_event(c);
            ev.b = get_event(c);
            DSCE_HIP_CHECK(hipEventRecord(ev.a, st));
        }
    }
    ~Timed() {
        if (on) {
            (void)hipEventRecord(ev.b, st);
            c->pending.push_back(ev);
        }
    }
};

void collect_timing(dsce_ctx* c) {
    for (auto& e : c->pending) {
        float ms = 0.f;
        DSCE_HIP_CHECK(hipEventElapsedTime(&ms, e.a, e.b));
        auto& t = c->ktime[e.name];
        t.first += 1;
        t.second += ms;
        c->event_pool.push_back(e.a);
        c->event_pool.push_back(e.b);
    }
    c->pending.clear();
}

Band upload_band(dsce_ctx* c, const HostBand& h, bool with_vals) {
    Band b{};
    b.nblk = (int)h.row0.size();
    b.rb = h.rb;
    b.row0 = dupload(c, h.row0);
    b.nrows = dupload(c, h.nrows);
    b.klo = dupload(c, h.klo);
    b.khi = dupload(c, h.khi);
    b.off = dupload(c, h.off);
    b.vals = with_vals ? dupload(c, h.vals) : nullptr;
    return b;
}

void check_ctx(dsce_ctx* c) {
    if (!c) throw ApiError(DSCE_EINVAL, "null context");
    DSCE_HIP_CHECK(hipSetDevice(c->device));
    // errors are per call: a failure some earlier call already returned (or a
    // teardown ignored) must not be reported again by this call's hipGetLastError
    // (every entry point checks its own launches at API_END, so a stale error here
    // comes from outside the engine; reported only with DSCE_DEBUG set)
    const hipError_t stale = hipGetLastError();
    if (stale != hipSuccess && getenv("DSCE_DEBUG"))
        fprintf(stderr, "dsce: clearing a stale HIP error at entry: %s\n", hipGetErrorString(stale));
}

Scheme& get_scheme(dsce_ctx* c, int id) {
    if (id < 0 || id >= (int)c->schemes.size()) throw ApiError(DSCE_EINVAL, "bad scheme id");
    return *c->schemes[id];
}

// ---------------------------------------------------------------------------
// Polyphase form of G and Q (SchemeK::poly_ok; the perfect-CSI IC passes
// k_poly_syn / k_poly_chan / k_poly_ana).  M = G or Q (N x LK, column l + L k):
// every symbol's columns are one real window times the subcarrier tones,
//   M[n, l + L k] = A_k[n] w^(l n) C[l][k],   w = e^(2 pi i / L)
// (FBMC: Hermite prototype p(t - k T/2) times e^(i 2 pi l F (t - k T/2)) and the
// OQAM phase, FBMC.m:255-285 / :318-354; OFDM: its CP / FFT window, OFDM.m:153-218).
// A_k is column 0 with its largest entry's phase removed, C follows from that
// entry; the factorisation is then checked on every entry of M.  Returns the
// largest |M - A w C| / max |M| (2 if a window is not real).
// ---------------------------------------------------------------------------
double poly_factor(const std::vector<double2>& M, int N, int L, int K, std::vector<double>& A,
                   std::vector<double2>& C) {
    A.assign((size_t)K * N, 0.0);
    C.assign((size_t)K * L, make_double2(0, 0));
    std::vector<double2> wt(L);
    for (int e = 0; e < L; ++e) wt[e] = make_double2(std::cos(2.0 * M_PI * e / L), std::sin(2.0 * M_PI * e / L));
    double mmax = 0.0;
    for (auto& z : M) mmax = std::max(mmax, std::hypot(z.x, z.y));
    if (!(mmax > 0.0)) return 2.0;
    double worst = 0.0;
    for (int k = 0; k < K; ++k) {
        const double2* c0 = &M[(size_t)(L * k) * N];
        int ns = 0;
        for (int n = 1; n < N; ++n)
            if (std::hypot(c0[n].x, c0[n].y) > std::hypot(c0[ns].x, c0[ns].y)) ns = n;
        const double g = std::hypot(c0[ns].x, c0[ns].y);
        if (!(g > 0.0)) return 2.0;
        const double2 ph = make_double2(c0[ns].x / g, -c0[ns].y / g);      // conj(c0[ns]) / |c0[ns]|
        for (int n = 0; n < N; ++n) {
            const double2 a = c_mul(c0[n], ph);
            if (std::fabs(a.y) > 1e-12 * mmax) return 2.0;
            A[(size_t)k * N + n] = a.x;
        }
        for (int l = 0; l < L; ++l) {
            const double2 wn = wt[(size_t)(((long long)l * ns) % L)];
            const double2 z = c_mul(M[(size_t)(l + L * k) * N + ns], make_double2(wn.x, -wn.y));
            C[(size_t)k * L + l] = make_double2(z.x / g, z.y / g);
        }
        for (int l = 0; l < L; ++l) {
            const double2 cl = C[(size_t)k * L + l];
            const double2* col = &M[(size_t)(l + L * k) * N];
            for (int n = 0; n < N; ++n) {
                const double2 wv = wt[(size_t)(((long long)l * n) % L)];
                const double2 f = c_scale(c_mul(wv, cl), A[(size_t)k * N + n]);
                worst = std::max(worst, std::hypot(col[n].x - f.x, col[n].y - f.y) / mmax);
            }
        }
    }
    return worst;
}

// SchemeK::poly_* from the host G and Q when both factorise to 1e-12 (the
// tolerance of the OFDM FFT form's check, pack_scheme) with F = L = 24 or 48
void build_poly(dsce_ctx* c, Scheme& s) {
    SchemeK& k = s.k;
    k.poly_ok = 0;
    const int N = s.N, L = s.d.n_subcarriers, K = s.d.n_symbols;
    if ((L != 24 && L != 48) || L * K != s.LK || N <= 0) return;
    const int ni = (N + L - 1) / L;
    if (ni > POLY_NI) return;
    std::vector<double> Ag, Aq;
    std::vector<double2> Cg, Cq;
    const double rg = poly_factor(s.G, N, L, K, Ag, Cg);
    const double rq = poly_factor(s.Q, N, L, K, Aq, Cq);
    s.poly_resid = std::max(rg, rq);
    if (!(s.poly_resid <= 1e-12)) return;
    // per residue m: the windows at n = m + L j, zero past N
    // (the A rows carry a leading zero: k_poly_chan's halves read j = i0 - 1 ..)
    std::vector<double> pa((size_t)L * K * POLY_NA, 0.0), pb((size_t)L * K * POLY_NI, 0.0);
    for (int m = 0; m < L; ++m)
        for (int kk = 0; kk < K; ++kk)
            for (int j = 0; j < POLY_NI; ++j) {
                const int n = m + L * j;
                if (n >= N) continue;
                pa[((size_t)m * K + kk) * POLY_NA + j + 1] = Ag[(size_t)kk * N + n];
                pb[((size_t)m * K + kk) * POLY_NI + j] = Aq[(size_t)kk * N + n];
            }
    // Q^H[l + L k, n] = conj(Q) = B_k[n] w^(-l n) conj(Cq[l][k]): E = conj(Cq)
    std::vector<double2> E(Cq.size());
    for (size_t i = 0; i < Cq.size(); ++i) E[i] = make_double2(Cq[i].x, -Cq[i].y);
    std::vector<double2> tw(L);
    for (int e = 0; e < L; ++e) tw[e] = make_double2(std::cos(2.0 * M_PI * e / L), std::sin(2.0 * M_PI * e / L));
    s.poly_nnz_a = s.poly_nnz_b = 0.0;
    for (size_t i = 0; i < Ag.size(); ++i) {
        s.poly_nnz_a += Ag[i] != 0.0;
        s.poly_nnz_b += Aq[i] != 0.0;
    }
    k.poly_F = L;
    k.poly_K = K;
    k.poly_ni = ni;
    k.poly_C = dupload(c, Cg);
    k.poly_E = dupload(c, E);
    k.poly_A = dupload(c, pa);
    k.poly_B = dupload(c, pb);
    k.poly_tw = dupload(c, tw);
    k.poly_ok = 1;
}

// The chain kernels' LDS tables (SchemeK::ct_*), evaluated with the kernels'
// own operations in the same order (the host code is built with
// -ffp-contract=off like the kernels, std::fma where they use fma), so the
// staged values are bit-identical to what each block derived from its thread
// index before r06.
static const double kW24h[12][2] = {
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

static double2 w24_signed(int e) {                 // w24^e, e in 0..23, as kW24[e % 12] negated past 12
    const double2 t = make_double2(kW24h[e % 12][0], kW24h[e % 12][1]);
    return e >= 12 ? make_double2(-t.x, -t.y) : t;
}

void build_chain_tables(dsce_ctx* c, Scheme& s, const std::vector<int>& grid, const std::vector<int>& row_data,
                        const std::vector<int>& row_cons, const std::vector<int>& row_pcol,
                        const std::vector<double2>& row_pval) {
    SchemeK& k = s.k;
    const int LK = s.LK, NP = s.d.n_pilots, M = s.d.mod_order;
    const double2 scale = k.pf_scale;
    const double cs = (1.0 / k.data_div) * k.slI;             // chain_detect's scI
    std::vector<double2> symc(256), sym(256), amt(192), twa(48), rpv, wrow;
    std::vector<int> rdc, rpc;
    for (int t = 0; t < 256; ++t) {
        const double2 a = t < M ? s.symbols[t] : make_double2(0.0, 0.0);
        double2 sa = a;
        if (k.pv_uni) {                                         // stage_sym: c_fma(0, pv, a)
            const double2 pv = k.pv_data;
            double x = std::fma(pv.x, a.x, 0.0);
            x = std::fma(-pv.y, a.y, x);
            double y = std::fma(pv.x, a.y, 0.0);
            y = std::fma(pv.y, a.x, y);
            sa = make_double2(x, y);
        }
        sym[t] = sa;
        symc[t] = make_double2(sa.x * cs, sa.y * cs);
    }
    for (int t = 0; t < 192; ++t) {                             // amt[dir][m][i + 4 k]
        const int dir = t / 96, m = (t / 16) % 6, ii = t & 3, kk = (t >> 2) & 3;
        const double2 v = w24_signed((6 * ii * kk + (dir ? ii : kk) * m) % 24);
        amt[t] = dir ? c_mul(scale, make_double2(v.x, -v.y)) : v;
    }
    for (int t = 0; t < 48; ++t) {                              // twa[dir][r][m']
        const double2 v = w24_signed(((t / 6) % 4) * (t % 6));
        twa[t] = t >= 24 ? c_mul(scale, make_double2(v.x, -v.y)) : v;
    }
    std::vector<unsigned> gw(64, 0u);
    for (int t = 0; t < 256; ++t) {
        const int gi = t >> 4, gq = t & 15;
        const unsigned g = gi < k.nI && gq < k.nQ ? (unsigned)grid[std::min(gi * k.nQ + gq, k.nI * k.nQ - 1)] & 0xffu : 0u;
        gw[t >> 2] |= g << (8 * (t & 3));
    }
    const size_t nblk = s.qband.row0.size();
    for (size_t b = 0; b < nblk; ++b)
        for (int rt = 0; rt < 24; ++rt) {
            const int r = std::min(s.qband.row0[b] + rt, LK - 1);
            const int dr = row_data[r], pc = row_pcol[r];
            rpv.push_back(row_pval[r]);
            rdc.push_back(dr >= 0 ? (dr << 1) | (row_cons[r] ? 1 : 0) : -1);
            rpc.push_back(dr < 0 && pc >= 0 && pc < NP ? pc : -1);
            const double2 wl = w24_signed(rt);
            wrow.push_back(c_mul(scale, make_double2(wl.x, -wl.y)));
        }
    k.ct_symc = dupload(c, symc);
    k.ct_sym = dupload(c, sym);
    k.ct_amt = dupload(c, amt);
    k.ct_twa = dupload(c, twa);
    k.ct_grid = dupload(c, gw);
    k.ct_rpv = dupload(c, rpv);
    k.ct_rdc = dupload(c, rdc);
    k.ct_rpc = dupload(c, rpc);
    k.ct_wrow = dupload(c, wrow);
}

// ---------------------------------------------------------------------------
// operator packing
// ---------------------------------------------------------------------------
void pack_scheme(dsce_ctx* c, Scheme& s) {
    const int N = s.N, LK = s.LK, Nsym = s.d.n_tx_symbols;
    // column supports (first/last non-zero sample) of G and Q
    std::vector<int> gs(LK), ge(LK), qs(LK), qe(LK);
    for (int col = 0; col < LK; ++col) {
        int a = N, b = -1, qa = N, qb = -1;
        for (int n = 0; n < N; ++n) {
            if (nz(s.G[(size_t)col * N + n])) { a = std::min(a, n); b = n; }
            if (nz(s.Q[(size_t)col * N + n])) { qa = std::min(qa, n); qb = n; }
        }
        if (b < 0) { a = 0; b = -1; }
        if (qb < 0) { qa = 0; qb = -1; }
        gs[col] = a; ge[col] = b; qs[col] = qa; qe[col] = qb;
    }
    s.GL = 1;
    s.QL = 1;
    for (int col = 0; col < LK; ++col) {
        s.GL = std::max(s.GL, ge[col] - gs[col] + 1);
        s.QL = std::max(s.QL, qe[col] - qs[col] + 1);
    }
    s.g_start = gs;
    s.q_start = qs;
    std::vector<double2> gcol((size_t)LK * s.GL, make_double2(0, 0)), qcol((size_t)LK * s.QL, make_double2(0, 0));
    for (int col = 0; col < LK; ++col) {
        for (int i = 0; i < s.GL && gs[col] + i < N; ++i) gcol[(size_t)col * s.GL + i] = s.G[(size_t)col * N + gs[col] + i];
        for (int i = 0; i < s.QL && qs[col] + i < N; ++i) qcol[(size_t)col * s.QL + i] = s.Q[(size_t)col * N + qs[col] + i];
    }
    // G band: rows = samples, k = columns
    std::vector<int> rlo(N, 0), rhi(N, 0);
    for (int n = 0; n < N; ++n) {
        int lo = LK, hi = -1;
        for (int col = 0; col < LK; ++col)
            if (nz(s.G[(size_t)col * N + n])) { lo = std::min(lo, col); hi = col; }
        rlo[n] = hi < 0 ? 0 : lo;
        rhi[n] = hi < 0 ? 0 : hi + 1;
    }
    s.gband = band_geometry(N, [&](int r, int& a, int& b) { a = rlo[r]; b = rhi[r]; }, 1);
    s.gband.vals.assign(s.gband.elems, make_double2(0, 0));
    for (size_t blk = 0; blk < s.gband.row0.size(); ++blk)
        for (int rl = 0; rl < s.gband.nrows[blk]; ++rl)
            for (int k = s.gband.klo[blk]; k < s.gband.khi[blk]; ++k)
                s.gband.vals[s.gband.off[blk] + (size_t)(k - s.gband.klo[blk]) * DSCE_RB + rl] =
                    s.G[(size_t)k * N + s.gband.row0[blk] + rl];
    // Q^H band: rows = columns of Q, k = samples
    s.qband = band_geometry(LK, [&](int r, int& a, int& b) { a = qs[r]; b = qe[r] + 1; }, 1);
    s.qband.vals.assign(s.qband.elems, make_double2(0, 0));
    for (size_t blk = 0; blk < s.qband.row0.size(); ++blk)
        for (int rl = 0; rl < s.qband.nrows[blk]; ++rl)
            for (int k = s.qband.klo[blk]; k < s.qband.khi[blk]; ++k) {
                const double2 q = s.Q[(size_t)(s.qband.row0[blk] + rl) * N + k];
                s.qband.vals[s.qband.off[blk] + (size_t)(k - s.qband.klo[blk]) * DSCE_RB + rl] = make_double2(q.x, -q.y);
            }
    // diag(D) = diag(Q' H G) as a banded matvec over the channel taps, rows c,
    // k = n * ntap + tau:  h[c] = sum_k conj(Q[n,c]) G[n - d_tau, c] IR[tau][n]
    {
        const int nt = c->ch.ntap;
        s.hband = band_geometry(LK, [&](int r, int& a, int& b) { a = qs[r] * nt; b = (qe[r] + 1) * nt; }, 1);
        s.hband.vals.assign(s.hband.elems, make_double2(0, 0));
        for (size_t blk = 0; blk < s.hband.row0.size(); ++blk)
            for (int rl = 0; rl < s.hband.nrows[blk]; ++rl) {
                const int col = s.hband.row0[blk] + rl;
                for (int k = s.hband.klo[blk]; k < s.hband.khi[blk]; ++k) {
                    const int n = k / nt, m = n - c->ch.tap_delay[k % nt];
                    if (m < 0 || n >= N) continue;
                    const double2 q = s.Q[(size_t)col * N + n], g = s.G[(size_t)col * N + m];
                    s.hband.vals[s.hband.off[blk] + (size_t)(k - s.hband.klo[blk]) * DSCE_RB + rl] =
                        make_double2(q.x * g.x + q.y * g.y, q.x * g.y - q.y * g.x);
                }
            }
    }
    // Q^H row blocks with disjoint sample ranges (OFDM): the noise can be drawn
    // inside the Q^H pass (LoadNoisy) without drawing a sample twice
    {
        std::vector<int> seen(N, 0);
        bool disj = true;
        for (size_t b = 0; b < s.qband.row0.size() && disj; ++b)
            for (int n = s.qband.klo[b]; n < s.qband.khi[b]; ++n)
                if (seen[n]++) disj = false;
        s.k.qh_disjoint = disj ? 1 : 0;
    }
    // block-local perfect-CSI IC (SchemeK::pic_ok): every Q^H block reads only
    // samples whose G columns are the block's own rows
    {
        int md = 0;
        for (int q = 0; q < c->ch.ntap; ++q) md = std::max(md, c->ch.tap_delay[q]);
        const int nb = (int)s.qband.row0.size();
        bool ok = true;
        for (int b = 0; b < nb && ok; ++b) {
            const int r0 = s.qband.row0[b], klo = s.qband.klo[b], khi = s.qband.khi[b];
            const int s0 = std::max(0, klo - md);
            for (int n = s0; n < khi && ok; ++n)
                for (int col = 0; col < LK && ok; ++col)
                    if (nz(s.G[(size_t)col * N + n]) && (col < r0 || col >= r0 + DSCE_RB)) ok = false;
        }
        s.k.pic_ok = ok && nb > 0 ? 1 : 0;
        // FFT form (SchemeK::pf_ok): 24-row blocks, 24-sample windows, G / Q^H
        // equal to gs w^(l m) / qs w^(-l m) (w = e^(2 pi i / 24), m = n - klo) to
        // 1e-12 relative, and the md samples before the window a cyclic prefix
        bool fok = s.k.pic_ok && md <= 1 && nb > 0;
        double2 gsc = make_double2(0, 0), qsc = make_double2(0, 0);
        if (fok) {
            gsc = s.G[(size_t)s.qband.row0[0] * N + s.qband.klo[0]];
            qsc = s.qband.vals[s.qband.off[0]];
            fok = std::hypot(gsc.x, gsc.y) > 0 && std::hypot(qsc.x, qsc.y) > 0;
        }
        const double gm = std::hypot(gsc.x, gsc.y), qm = std::hypot(qsc.x, qsc.y);
        for (int b = 0; b < nb && fok; ++b) {
            const int r0 = s.qband.row0[b], klo = s.qband.klo[b], khi = s.qband.khi[b];
            if (s.qband.nrows[b] != 24 || khi - klo != 24 || klo - md < 0 || r0 + 24 > LK) {
                fok = false;
                break;
            }
            for (int lr = 0; lr < 24 && fok; ++lr)
                for (int m = -md; m < 24 && fok; ++m) {
                    const int e = (((lr * m) % 24) + 24) % 24;
                    const double ang = 2.0 * M_PI * e / 24.0;
                    const double2 wv = make_double2(std::cos(ang), std::sin(ang));
                    const double2 gmod = make_double2(gsc.x * wv.x - gsc.y * wv.y, gsc.x * wv.y + gsc.y * wv.x);
                    const double2 gv = s.G[(size_t)(r0 + lr) * N + klo + m];
                    if (std::hypot(gv.x - gmod.x, gv.y - gmod.y) > 1e-12 * gm) fok = false;
                    if (m < 0) continue;
                    const double2 qmod = make_double2(qsc.x * wv.x + qsc.y * wv.y, qsc.y * wv.x - qsc.x * wv.y);
                    const double2 qv = s.qband.vals[s.qband.off[b] + (size_t)m * DSCE_RB + lr];
                    if (std::hypot(qv.x - qmod.x, qv.y - qmod.y) > 1e-12 * qm) fok = false;
                }
        }
        s.k.pf_ok = fok ? 1 : 0;
        s.k.pf_scale = make_double2(qsc.x * gsc.x - qsc.y * gsc.y, qsc.x * gsc.y + qsc.y * gsc.x);
        s.k.pf_gs = gsc;
        s.k.pf_qs = qsc;
    }
    // W band: rows r, k = (c, p); c overlaps where Q-support(r) meets (H G)-support(c)
    int maxd = 0;
    for (int q = 0; q < c->ch.ntap; ++q) maxd = std::max(maxd, c->ch.tap_delay[q]);
    s.maxdelay = maxd;
    const int NP = s.d.n_pilots;
    s.wband = band_geometry(
        LK,
        [&](int r, int& a, int& b) {
            a = LK;
            b = -1;
            for (int col = 0; col < LK; ++col) {
                if (qe[r] < qs[r] || ge[col] < gs[col]) continue;
                if (gs[col] <= qe[r] && qs[r] <= ge[col] + maxd) { a = std::min(a, col); b = col + 1; }
            }
            if (b < 0) { a = 0; b = 0; }
        },
        NP, DSCE_WRB, true);
    s.w_elems = s.wband.elems;
    band_work(s.wband, NP, s.w_struct, s.w_diag);
    // precoder CSR and its conjugate transpose
    std::vector<int> pptr(LK + 1, 0), pcol;
    std::vector<double2> pval;
    for (int r = 0; r < LK; ++r) {
        for (int k = 0; k < Nsym; ++k) {
            const double2 v = s.P[(size_t)k * LK + r];
            if (nz(v)) { pcol.push_back(k); pval.push_back(v); }
        }
        pptr[r + 1] = (int)pcol.size();
    }
    std::vector<int> hptr(Nsym + 1, 0), hcol;
    std::vector<double2> hval;
    for (int k = 0; k < Nsym; ++k) {
        for (int r = 0; r < LK; ++r) {
            const double2 v = s.P[(size_t)k * LK + r];
            if (nz(v)) { hcol.push_back(r); hval.push_back(make_double2(v.x, -v.y)); }
        }
        hptr[k + 1] = (int)hcol.size();
    }
    // slicer grid of the constellation
    std::vector<double> lvI, lvQ;
    for (auto& z : s.symbols) { lvI.push_back(z.x); lvQ.push_back(z.y); }
    std::sort(lvI.begin(), lvI.end());
    lvI.erase(std::unique(lvI.begin(), lvI.end()), lvI.end());
    std::sort(lvQ.begin(), lvQ.end());
    lvQ.erase(std::unique(lvQ.begin(), lvQ.end()), lvQ.end());
    if ((int)(lvI.size() * lvQ.size()) != s.d.mod_order)
        throw ApiError(DSCE_EINVAL, "constellation is not a full rectangular grid");
    std::vector<int> grid(lvI.size() * lvQ.size(), -1);
    for (int m = 0; m < s.d.mod_order; ++m) {
        const int iI = (int)(std::lower_bound(lvI.begin(), lvI.end(), s.symbols[m].x) - lvI.begin());
        const int iQ = (int)(std::lower_bound(lvQ.begin(), lvQ.end(), s.symbols[m].y) - lvQ.begin());
        grid[(size_t)iI * lvQ.size() + iQ] = m;
    }
    // kernel view
    SchemeK& k = s.k;
    k.N = N;
    k.LK = LK;
    k.Nsym = Nsym;
    k.NP = NP;
    k.ND = s.d.n_data;
    k.M = s.d.mod_order;
    k.mbits = s.d.bits_per_symbol;
    k.despread = s.d.despread;
    k.real_detect = s.d.real_detect;
    k.inv_sqrt_kappa = 1.0 / sqrt(s.d.kappa);
    k.data_div = s.d.data_div;
    k.pilot_pos = dupload(c, s.pilot_pos);
    k.data_pos = dupload(c, s.data_pos);
    k.considered = dupload(c, std::vector<int>(s.considered.begin(), s.considered.end()));
    k.symbols = dupload(c, s.symbols);
    k.nI = (int)lvI.size();
    k.nQ = (int)lvQ.size();
    k.lvI = dupload(c, lvI);
    k.lvQ = dupload(c, lvQ);
    k.grid_sym = dupload(c, grid);
    k.slI = lvI.size() > 1 ? 1.0 / (lvI[1] - lvI[0]) : 1.0;
    k.slQ = lvQ.size() > 1 ? 1.0 / (lvQ[1] - lvQ[0]) : 1.0;
    k.lv0I = lvI.empty() ? 0.0 : lvI[0];
    k.lv0Q = lvQ.empty() ? 0.0 : lvQ[0];
    k.p_ptr = dupload(c, pptr);
    k.p_col = dupload(c, pcol);
    k.p_val = dupload(c, pval);
    k.ph_ptr = dupload(c, hptr);
    k.ph_col = dupload(c, hcol);
    k.ph_val = dupload(c, hval);
    k.G = upload_band(c, s.gband, true);
    k.QH = upload_band(c, s.qband, true);
    k.HD = upload_band(c, s.hband, true);
    k.q_start = dupload(c, qs);
    k.q_col = dupload(c, qcol);
    k.QL = s.QL;
    k.g_start = dupload(c, gs);
    k.g_col = dupload(c, gcol);
    k.GL = s.GL;
    s.wband_struct = s.wband;
    s.Wb = upload_band(c, s.wband, false);
    build_poly(c, s);
    // fused-stage maps (select mode): data index per row; row-local precoder
    {
        std::vector<int> row_data(LK, -1), row_pcol(LK, -1);
        std::vector<double2> row_pval(LK, make_double2(0.0, 0.0));
        if (!s.d.despread)
            for (int i = 0; i < s.d.n_data; ++i) row_data[s.data_pos[i]] = i;
        bool diag = !s.d.despread;
        for (int r = 0; r < LK && diag; ++r) {
            if (pptr[r + 1] - pptr[r] > 1) diag = false;
            else if (pptr[r + 1] == pptr[r] + 1) {
                const int kc = pcol[pptr[r]];
                if (kc >= NP && s.data_pos[kc - NP] != r) diag = false;
                row_pcol[r] = kc;
                row_pval[r] = pval[pptr[r]];
            }
        }
        std::vector<int> row_cons(LK, 0);
        for (int r = 0; r < LK; ++r)
            if (row_data[r] >= 0) row_cons[r] = s.considered[row_data[r]] ? 1 : 0;
        s.k.row_data = dupload(c, row_data);
        s.k.row_cons = dupload(c, row_cons);
        s.k.row_pcol = dupload(c, row_pcol);
        s.k.row_pval = dupload(c, row_pval);
        s.k.p_diag = diag ? 1 : 0;
        {
            bool uni = diag, first = true;
            double2 pv0 = make_double2(0.0, 0.0);
            for (int r = 0; r < LK && uni; ++r) {
                if (row_data[r] < 0) continue;
                if (first) pv0 = row_pval[r], first = false;
                else if (row_pval[r].x != pv0.x || row_pval[r].y != pv0.y) uni = false;
            }
            s.k.pv_uni = uni && !first ? 1 : 0;
            s.k.pv_data = pv0;
        }
        {
            std::vector<int> seen((size_t)NP + s.d.n_data, 0);
            for (int r = 0; r < LK; ++r)
                if (row_pcol[r] >= 0 && row_pcol[r] < NP + s.d.n_data) ++seen[row_pcol[r]];
            bool onto = diag;
            for (int v : seen) onto = onto && v == 1;
            s.k.tx_rows = onto ? 1 : 0;
        }
        if (s.k.pf_ok) build_chain_tables(c, s, grid, row_data, row_cons, row_pcol, row_pval);
    }
    // bits per realisation
    s.bits_all = (int64_t)s.d.n_data * s.d.bits_per_symbol;
    int64_t ce = 0;
    for (auto v : s.considered) ce += v ? 1 : 0;
    s.bits_noedge = ce * s.d.bits_per_symbol;
}

// ---------------------------------------------------------------------------
// Trim every W block to the column range that holds a non-zero entry in some
// (variant, SNR) slice after the 1e-8 threshold, and repack.  The contraction
// only skips exact zeros, so results are bit-identical; at C3/C4 the thresholded
// estimator spans |dk| <= 7 symbols instead of the structural 15.
// ---------------------------------------------------------------------------
void trim_w_band(dsce_ctx* c, Scheme& s, std::vector<void*>& tmp) {
    if (!c->op.wtrim) return;                    // Opts::wtrim = 0 keeps the structural band
    hipStream_t st = c->stream;
    const int NP = s.d.n_pilots, nsl = 2 * c->nsnr, nblk = (int)s.wband.row0.size();
    int* dlohi;
    DSCE_HIP_CHECK(hipMalloc(&dlohi, 2 * nblk * sizeof(int)));
    tmp.push_back(dlohi);
    std::vector<int> lohi(2 * nblk);
    for (int b = 0; b < nblk; ++b) {
        lohi[2 * b] = 1 << 30;
        lohi[2 * b + 1] = -1;
    }
    DSCE_HIP_CHECK(hipMemcpy(dlohi, lohi.data(), lohi.size() * sizeof(int), hipMemcpyHostToDevice));
    setup_w_extent(st, s.Wb, NP, s.W, s.w_elems, nsl, dlohi);
    DSCE_HIP_CHECK(hipMemcpyAsync(lohi.data(), dlohi, lohi.size() * sizeof(int), hipMemcpyDeviceToHost, st));
    DSCE_HIP_CHECK(hipStreamSynchronize(st));
    HostBand nb = s.wband;
    nb.vals.clear();
    long long off = 0;
    for (int b = 0; b < nblk; ++b) {
        const int clo = s.wband.klo[b] / NP;
        int lo = lohi[2 * b], hi = lohi[2 * b + 1];
        if (hi < lo) { lo = 0; hi = -1; }
        nb.klo[b] = (clo + lo) * NP;
        nb.khi[b] = (clo + hi + 1) * NP;
        nb.off[b] = off;
        off += (long long)(hi - lo + 1) * NP * nb.rb;
    }
    nb.elems = off;
    if (off == s.w_elems) return;
    double2* W2 = dalloc<double2>(c, (size_t)nsl * std::max<long long>(off, 1));
    for (int sl = 0; sl < nsl; ++sl)
        for (int b = 0; b < nblk; ++b) {
            const long long n = (long long)(nb.khi[b] - nb.klo[b]) * nb.rb;
            if (n == 0) continue;
            const long long src = s.wband.off[b] + (long long)(nb.klo[b] - s.wband.klo[b]) * nb.rb;
            DSCE_HIP_CHECK(hipMemcpyAsync(W2 + (size_t)sl * off + nb.off[b], s.W + (size_t)sl * s.w_elems + src,
                                          n * sizeof(double2), hipMemcpyDeviceToDevice, st));
        }
    DSCE_HIP_CHECK(hipStreamSynchronize(st));
    free_alloc(c, s.W);          // release the untrimmed estimator and switch geometry
    s.W = W2;
    s.wband = nb;
    s.w_elems = off;
    band_work(nb, NP, s.w_struct, s.w_diag);
    s.Wb = upload_band(c, nb, false);
}

// ---------------------------------------------------------------------------
// setup pipeline: R_hP, R_est, R_noI, R_Dij, W, W0 (script:208-313)
// Pair-tile copy of the trimmed W band for k_wpair3 (NP a multiple of 4 with
// NP/4 in {2, 4, 8}; 24-row pair blocks when every block has <= 24 rows, else 32).
void build_wpair(dsce_ctx* c, Scheme& s) {
    const int NP = s.d.n_pilots, nblk = (int)s.wband.row0.size();
    if (NP % 4 != 0 || (NP / 4 != 2 && NP / 4 != 4 && NP / 4 != 8)) return;
    int maxrows = 0;
    for (int b = 0; b < nblk; ++b) maxrows = std::max(maxrows, s.wband.nrows[b]);
    if (maxrows > 32) return;
    const int rbp = maxrows <= 24 ? 24 : 32;
    std::vector<int> row0(nblk), nrows(nblk), clo(nblk), ntile(nblk);
    std::vector<long long> off(nblk);
    long long o = 0, exec = 0;
    for (int b = 0; b < nblk; ++b) {
        row0[b] = s.wband.row0[b];
        nrows[b] = s.wband.nrows[b];
        clo[b] = s.wband.klo[b] / NP;
        int ncol = (s.wband.khi[b] - s.wband.klo[b]) / NP;
        if (rbp == 24) ncol += ncol & 1;                 // tiles come in periods of 3 (2 columns)
        ntile[b] = ncol * rbp / 16;
        off[b] = o;
        o += (long long)ntile[b] * NP * 16;
        exec += (long long)ntile[b] * 16 * NP;
    }
    s.Pb.nblk = nblk;
    s.Pb.rbp = rbp;
    s.Pb.nks = NP / 4;
    s.Pb.row0 = dupload(c, row0);
    s.Pb.nrows = dupload(c, nrows);
    s.Pb.clo = dupload(c, clo);
    s.Pb.ntile = dupload(c, ntile);
    s.Pb.off = dupload(c, off);
    s.wp_elems = std::max<long long>(o, 1);
    s.wp_exec = exec;
    const int nsl = 2 * c->nsnr;
    // the complex pair tiles are only the packer's intermediate: freed once the
    // 3M planes exist
    double2* wp = dalloc<double2>(c, (size_t)nsl * s.wp_elems);
    // W's 3M planes, two k-steps per 16-byte lane load
    s.Wp3 = dalloc<double>(c, (size_t)nsl * 3 * s.wp_elems);
    setup_wpair(c->stream, s.Wb, NP, s.W, s.w_elems, s.Pb, wp, s.wp_elems, nsl, s.Wp3);
    free_alloc(c, wp);
    // fused MMSE stage: block-diagonal W (every block's columns are its own 24
    // rows, OFDM), row-local precoder, select-mode detection, NP = 16
    bool fuse = rbp == 24 && NP == 16 && s.k.p_diag && !s.d.despread;
    for (int b = 0; b < nblk && fuse; ++b)
        if (nrows[b] != 24 || s.wband.klo[b] / NP < row0[b] || s.wband.khi[b] / NP > row0[b] + 24) fuse = false;
    if (fuse) {
        std::vector<int> pblk(NP), pc0(NP);
        for (int i = 0; i < NP; ++i) {
            const int r = s.pilot_pos[i];
            int bb = -1;
            for (int b = 0; b < nblk; ++b)
                if (r >= row0[b] && r < row0[b] + nrows[b]) bb = b;
            if (bb < 0) fuse = false;
            pblk[i] = bb;
            pc0[i] = bb < 0 ? 0 : row0[bb];
        }
        if (fuse) {
            int* dpb = dupload(c, pblk);
            int* dpp = dupload(c, s.pilot_pos);
            s.pil_c0 = dupload(c, pc0);
            s.Wpil = dalloc<double2>(c, (size_t)nsl * NP * 24 * NP);
            s.WdA = dalloc<double2>(c, (size_t)nsl * nblk * 2 * (NP / 4) * 64);
            setup_fused_stage(c->stream, s.Wb, s.LK, NP, s.W, s.w_elems, s.Wd, nsl, dpb, dpp, 24, s.Wpil, s.WdA);
            DSCE_HIP_CHECK(hipStreamSynchronize(c->stream));
            DSCE_HIP_CHECK(hipGetLastError());
            free_alloc(c, dpb);
            free_alloc(c, dpp);
        }
    }
}

// ---------------------------------------------------------------------------
// Interpolation estimator (dsce_set_interpolation): the one-tap channel of every
// stage is I hP, held in the Wd slots [var][snr] so the stage kernels and
// dsce_mmse_onetap use it unchanged; there is no W, so no IC iterations.
void upload_interp(dsce_ctx* c, Scheme& s) {
    if (s.Wd) free_alloc(c, s.Wd);
    s.Wd = nullptr;
    const int nsl = 2 * std::max(c->nsnr, 1);
    std::vector<double2> rep((size_t)nsl * s.interp_I.size());
    for (int i = 0; i < nsl; ++i) std::copy(s.interp_I.begin(), s.interp_I.end(), rep.begin() + (size_t)i * s.interp_I.size());
    s.Wd = dupload(c, rep);
    s.mmse_ready = c->nsnr > 0;
}

// ---------------------------------------------------------------------------
// Operator of the structured MMSE IC (k_mic_pilot / k_mic_data): D_hat = Q' H_hat G with the
// estimated taps H_hat = Bv hP (setup_bv).  Eligible: FFT-form OFDM blocks
// (SchemeK::pf_ok), the fused stage's pilot pre-pass (Wpil), NP = 16, at most two
// taps with delays <= 1.  Kept only if Q' H_hat G reproduces EVERY entry of the
// thresholded W of every (variant, SNR) slice — the diagonal (Wd, the one-tap
// channel of script:428/:515) and the off-diagonal entries the IC subtraction
// uses (the packed band, script:482-484), zero across FFT blocks — to rounding:
// |difference| <= rtol max|W| per entry, rtol = max(MIC_RTOL, LR_EPS kappa(R)) of
// the slice (capped at MIC_RTOL_MAX; kappa(R) = ||R||_1 ||pinv(R)||_1: W and Bv
// both carry rounding of order eps kappa(R) through pinv(R)).  That is the check that the
// sparsification of R_Dij,hP and W (script:264-265, :287-289, :306-308) drops
// nothing but rounding-level entries: an entry the threshold zeroed has
// |W_s| < thr, so a guard at thr (r02-r03: thr + 1e-9 max|W|) would accept any
// geometry whose only deviation is the threshold itself.
// C2 at the script's 1e-8: 7e-13 absolute, max|W| 0.41-0.59 (tools/threshold_study.py).
//
// In FFT form block b of Q' H_hat_p G is, with w = e^(2 pi i / 24), m = n - klo_b,
//   D_p[lr, lc] = qs gs sum_q w^(-lc d_q) F_q[lc - lr],  F_q[k] = sum_m w^(k m) Bv[q][klo_b + m][p]
// (Q^H row lr = qs w^(-lr m), G column lc = gs w^(lc m), cyclic over the prefix).
// The low-rank form of the structured MMSE IC operator (Opts::mic_lr).  For
// OFDM the pilot columns of Q and G are one FFT window's exponentials, so
// Q[b + d_q, j] conj(G[b, j]) is a constant over pilot j's window and k_mcoef's
// m[j][q][n - d_q] = kappa_qj T_{k(j)}[n] with T_k[n] = sum_{b in W_k} J0(n - b)
// the J0 kernel summed over the FFT window W_k of pilot symbol k, for every tap.
// Hence Bv[q][n][p] = sum_k T_k[n] Bz[q k][p], Bz[q k][p] = sum_{j in W_k}
// kappa_qj pinv(R)[j][p]: the estimated taps of a symbol are MIC_NB real x
// complex MACs per tap and sample from Z = Bz hP (NT MIC_NB x NP complex MACs per
// unit and stage, shared by every symbol) instead of NP complex MACs from hP.
// Bz is fitted here to the Bv the guard above checked (least squares over every
// FFT-window sample, long-double QR of the MIC_NB columns of T) and kept only if
// the fit reproduces Bv to rounding in every (variant, SNR) slice:
// max |Bv - T Bz| <= min(MIC_RTOL_MAX, max(1e-13, LR_EPS kappa(R))) max |Bv| with kappa(R) =
// ||R||_1 ||pinv(R)||_1 — the GPU's Bv = m pinv(R) itself carries rounding of
// that order (the oracle's C2 fit: 8.6e-15 at cond 1.1e2 up to 7.2e-12 at
// cond 1.2e5, tests/test_lowrank.py), while a geometry without the structure
// misses by orders of magnitude.
static constexpr double LR_EPS = 4e-16;
// the structured-OFDM guards' per-slice bars (build_mic, build_mic_lr): at least
// MIC_RTOL, at most MIC_RTOL_MAX, relative to max|W| / max|Bv|
static constexpr double MIC_RTOL = 1e-11, MIC_RTOL_MAX = 1e-9;
// max(column, row) 1-norm of an NP x NP complex matrix (its condition estimate
// kappa(R) = ||R||_1 ||pinv(R)||_1 sets the rounding bars of build_mic / build_mic_lr)
double norm1(const double2* m, int NP) {
    double best = 0.0;
    for (int j = 0; j < NP; ++j) {
        double cs = 0.0, rs = 0.0;
        for (int i = 0; i < NP; ++i) {
            cs += std::hypot(m[(size_t)j * NP + i].x, m[(size_t)j * NP + i].y);
            rs += std::hypot(m[(size_t)i * NP + j].x, m[(size_t)i * NP + j].y);
        }
        best = std::max(best, std::max(cs, rs));
    }
    return best;
}
// R of slice sl = var nsnr + snr (R_est for var 0, R_noI for var 1)
const double2* slice_R(const Scheme& s, int nsnr, int sl) {
    const int NP = s.d.n_pilots;
    return sl < nsnr ? s.R_est.data() + (size_t)sl * NP * NP : s.R_noI.data() + (size_t)(sl - nsnr) * NP * NP;
}
void build_mic_lr(dsce_ctx* c, Scheme& s, const SetupArgs& a, const std::vector<double2>& bv, const std::vector<int>& pb,
                  const double2* rinv_dev) {
    const int NP = s.d.n_pilots, N = s.N, nt = c->ch.ntap, nsl = 2 * c->nsnr, nblk = s.k.QH.nblk;
    if ((int)pb.size() != MIC_NB || nt > 2) return;
    std::vector<double> j0((size_t)2 * N - 1);
    DSCE_HIP_CHECK(hipMemcpy(j0.data(), a.j0tab, j0.size() * sizeof(double), hipMemcpyDeviceToHost));
    // rows: every FFT-window sample of the scheme's blocks
    std::vector<int> rows;
    for (int b = 0; b < nblk; ++b)
        for (int m = 0; m < 24; ++m) rows.push_back(s.qband.klo[b] + m);
    const int nr = (int)rows.size();
    auto Tk = [&](int k, int n) {
        long double t = 0.0L;
        const int w0 = s.qband.klo[pb[k]];
        for (int m = 0; m < 24; ++m) t += (long double)j0[(size_t)(n - (w0 + m) + N - 1)];
        return t;
    };
    std::vector<long double> T((size_t)nr * MIC_NB);
    for (int i = 0; i < nr; ++i)
        for (int k = 0; k < MIC_NB; ++k) T[(size_t)i * MIC_NB + k] = Tk(k, rows[i]);
    // modified Gram-Schmidt QR of T (nr x MIC_NB)
    std::vector<long double> Qm(T), Rm(MIC_NB * MIC_NB, 0.0L);
    for (int k = 0; k < MIC_NB; ++k) {
        for (int j = 0; j < k; ++j) {
            long double d = 0.0L;
            for (int i = 0; i < nr; ++i) d += Qm[(size_t)i * MIC_NB + j] * Qm[(size_t)i * MIC_NB + k];
            Rm[j * MIC_NB + k] = d;
            for (int i = 0; i < nr; ++i) Qm[(size_t)i * MIC_NB + k] -= d * Qm[(size_t)i * MIC_NB + j];
        }
        long double nn = 0.0L;
        for (int i = 0; i < nr; ++i) nn += Qm[(size_t)i * MIC_NB + k] * Qm[(size_t)i * MIC_NB + k];
        nn = sqrtl(nn);
        if (!(nn > 0.0L)) return;
        Rm[k * MIC_NB + k] = nn;
        for (int i = 0; i < nr; ++i) Qm[(size_t)i * MIC_NB + k] /= nn;
    }
    // condition estimate of each slice's R: ||R||_1 ||pinv(R)||_1 (slice sl = var nsnr + snr)
    std::vector<double2> ri((size_t)nsl * NP * NP);
    DSCE_HIP_CHECK(hipMemcpy(ri.data(), rinv_dev, ri.size() * sizeof(double2), hipMemcpyDeviceToHost));
    std::vector<double2> bz((size_t)nsl * nt * MIC_NB * NP);
    double worst = 0.0, rel = 0.0;
    for (int sl = 0; sl < nsl; ++sl) {
        const double kap = norm1(slice_R(s, c->nsnr, sl), NP) * norm1(ri.data() + (size_t)sl * NP * NP, NP);
        // capped like build_mic's bar: a badly conditioned slice cannot
        // admit a fit above the rounding level the structured IC guard enforces
        const double tol = std::min(MIC_RTOL_MAX, std::max(1e-13, LR_EPS * kap));
        double mx = 0.0, dev = 0.0;
        for (int q = 0; q < nt; ++q)
            for (int p = 0; p < NP; ++p) {
                long double zr[MIC_NB], zi[MIC_NB];
                for (int k = 0; k < MIC_NB; ++k) {           // Q^T b
                    long double ar = 0.0L, ai = 0.0L;
                    for (int i = 0; i < nr; ++i) {
                        const double2 v = bv[(((size_t)sl * nt + q) * N + rows[i]) * NP + p];
                        ar += Qm[(size_t)i * MIC_NB + k] * v.x;
                        ai += Qm[(size_t)i * MIC_NB + k] * v.y;
                    }
                    zr[k] = ar;
                    zi[k] = ai;
                }
                for (int k = MIC_NB - 1; k >= 0; --k) {      // R z = Q^T b
                    for (int j = k + 1; j < MIC_NB; ++j) {
                        zr[k] -= Rm[k * MIC_NB + j] * zr[j];
                        zi[k] -= Rm[k * MIC_NB + j] * zi[j];
                    }
                    zr[k] /= Rm[k * MIC_NB + k];
                    zi[k] /= Rm[k * MIC_NB + k];
                }
                for (int k = 0; k < MIC_NB; ++k)
                    bz[(((size_t)sl * nt + q) * MIC_NB + k) * NP + p] = make_double2((double)zr[k], (double)zi[k]);
                for (int i = 0; i < nr; ++i) {
                    const double2 v = bv[(((size_t)sl * nt + q) * N + rows[i]) * NP + p];
                    long double er = -(long double)v.x, ei = -(long double)v.y;
                    for (int k = 0; k < MIC_NB; ++k) {
                        er += T[(size_t)i * MIC_NB + k] * (long double)(double)zr[k];
                        ei += T[(size_t)i * MIC_NB + k] * (long double)(double)zi[k];
                    }
                    dev = std::max(dev, (double)sqrtl(er * er + ei * ei));
                    mx = std::max(mx, std::hypot(v.x, v.y));
                }
            }
        if (!(mx > 0.0)) return;
        rel = std::max(rel, dev / mx);
        worst = std::max(worst, dev / (tol * mx));
    }
    s.lr_resid = rel;
    s.lr_ratio = worst;
    if (worst > 1.0) return;
    // Tw holds T_k minus its window mean (r06): the taps the IC stages form from
    // it, sum_k Tw_k Z[q k], are the estimated taps minus their window mean,
    // whose DFT-24 chain is exactly Q' H_hat G - diag(D_hat) (a constant tap over
    // the window maps to that diagonal), so y_ic = y - chain needs no
    // diag(D_hat) v term; Ts keeps the full window sums (diag(D_hat) itself)
    std::vector<double> tw((size_t)nblk * MIC_NB * 24), ts((size_t)nblk * MIC_NB);
    for (int b = 0; b < nblk; ++b)
        for (int k = 0; k < MIC_NB; ++k) {
            long double sum = 0.0L, t[24];
            for (int m = 0; m < 24; ++m) {
                t[m] = Tk(k, s.qband.klo[b] + m);
                sum += t[m];
            }
            for (int m = 0; m < 24; ++m) tw[((size_t)b * MIC_NB + k) * 24 + m] = (double)(t[m] - sum / 24.0L);
            ts[(size_t)b * MIC_NB + k] = (double)sum;
        }
    s.Bz = dupload(c, bz);
    s.Tw = dupload(c, tw);
    s.Ts = dupload(c, ts);
}

void build_mic(dsce_ctx* c, Scheme& s, const SetupArgs& a, const double2* m, const double2* rinv) {
    const int NP = s.d.n_pilots, LK = s.LK, N = s.N, nsl = 2 * c->nsnr, nt = c->ch.ntap;
    const int nblk = s.k.QH.nblk;
    bool ok = s.k.pf_ok && s.Wpil && NP == 16 && nt >= 1 && nt <= 2;
    for (int q = 0; q < nt && ok; ++q) ok = c->ch.tap_delay[q] <= 1;
    if (nt == 2 && ok) ok = c->ch.tap_delay[0] != c->ch.tap_delay[1];
    if (!ok) return;
    s.Bv = dalloc<double2>(c, (size_t)nsl * nt * s.N * NP);
    s.Bs = dalloc<double2>(c, (size_t)nsl * nblk * nt * NP);
    setup_bv(c->stream, a, nsl, m, rinv, s.Bv, nblk, s.k.QH.klo, 24, s.Bs);
    std::vector<double2> bv((size_t)nsl * nt * N * NP), wd((size_t)nsl * LK * NP), wb((size_t)nsl * s.w_elems);
    DSCE_HIP_CHECK(hipMemcpyAsync(bv.data(), s.Bv, bv.size() * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    DSCE_HIP_CHECK(hipMemcpyAsync(wd.data(), s.Wd, wd.size() * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    DSCE_HIP_CHECK(hipMemcpyAsync(wb.data(), s.W, wb.size() * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    DSCE_HIP_CHECK(hipStreamSynchronize(c->stream));
    const double2 ps = s.k.pf_scale;
    // FFT block of each row (-1: none)
    std::vector<int> fblk(LK, -1);
    for (int b = 0; b < nblk; ++b)
        for (int lr = 0; lr < 24; ++lr) fblk[s.qband.row0[b] + lr] = b;
    std::vector<double2> wpow(24);
    for (int e = 0; e < 24; ++e) wpow[e] = make_double2(std::cos(2.0 * M_PI * e / 24.0), std::sin(2.0 * M_PI * e / 24.0));
    const HostBand& wbnd = s.wband;
    // D[sl][b][p][lr][lc] of one slice at a time
    std::vector<double2> F((size_t)nt * 24), Ds((size_t)nblk * NP * 576);
    std::vector<char> seen((size_t)nblk * 576);
    std::vector<double2> ri((size_t)nsl * NP * NP);
    DSCE_HIP_CHECK(hipMemcpy(ri.data(), rinv, ri.size() * sizeof(double2), hipMemcpyDeviceToHost));
    double worst = 0.0, dev = 0.0, wmax = 0.0, rtol_max = MIC_RTOL;
    for (int sl = 0; sl < nsl; ++sl) {
        double mx = 0.0, md = 0.0;
        // the slice's rounding bar: W = R_Dij pinv(R) and Bv = m pinv(R) carry
        // rounding of order eps kappa(R) relative (GPU, C2: 5.9e-12 absolute at
        // max|W| 0.59 and kappa ~1e5), so max(MIC_RTOL, LR_EPS kappa(R)) max|W|
        // (capped at MIC_RTOL_MAX, a tenth of the script's threshold relative to |W| ~ 1)
        const double rtol = std::min(MIC_RTOL_MAX, std::max(MIC_RTOL, LR_EPS * norm1(slice_R(s, c->nsnr, sl), NP) *
                                                                           norm1(ri.data() + (size_t)sl * NP * NP, NP)));
        rtol_max = std::max(rtol_max, rtol);
        const double2* wds = wd.data() + (size_t)sl * LK * NP;
        const double2* wbs = wb.data() + (size_t)sl * s.w_elems;
        for (int i = 0; i < LK * NP; ++i) mx = std::max(mx, std::hypot(wds[i].x, wds[i].y));
        for (long long i = 0; i < s.w_elems; ++i) mx = std::max(mx, std::hypot(wbs[i].x, wbs[i].y));
        for (int b = 0; b < nblk; ++b) {
            const int klo = s.qband.klo[b];
            for (int p = 0; p < NP; ++p) {
                for (int q = 0; q < nt; ++q)
                    for (int k = 0; k < 24; ++k) {
                        double2 acc = make_double2(0, 0);
                        for (int mm = 0; mm < 24; ++mm)
                            acc = c_add(acc, c_mul(wpow[(k * mm) % 24],
                                                   bv[(((size_t)sl * nt + q) * N + klo + mm) * NP + p]));
                        F[(size_t)q * 24 + k] = acc;
                    }
                for (int lr = 0; lr < 24; ++lr)
                    for (int lc = 0; lc < 24; ++lc) {
                        double2 acc = make_double2(0, 0);
                        for (int q = 0; q < nt; ++q)
                            acc = c_add(acc, c_mul(wpow[(24 - (lc * c->ch.tap_delay[q]) % 24) % 24],
                                                   F[(size_t)q * 24 + (lc - lr + 24) % 24]));
                        Ds[((size_t)b * NP + p) * 576 + lr * 24 + lc] = c_mul(ps, acc);
                    }
            }
        }
        // diagonal: Wd
        for (int r = 0; r < LK; ++r) {
            const int b = fblk[r];
            for (int p = 0; p < NP; ++p) {
                const double2 ref = wds[(size_t)r * NP + p];
                double2 st = make_double2(0, 0);
                if (b >= 0) {
                    const int lr = r - s.qband.row0[b];
                    st = Ds[((size_t)b * NP + p) * 576 + lr * 24 + lr];
                }
                md = std::max(md, std::hypot(st.x - ref.x, st.y - ref.y));
            }
        }
        // off-diagonal: every entry of the (trimmed) band, then the in-block
        // pairs the band does not hold (W = 0 there)
        std::fill(seen.begin(), seen.end(), 0);
        for (size_t blk = 0; blk < wbnd.row0.size(); ++blk) {
            const int clo = wbnd.klo[blk] / NP, chi = wbnd.khi[blk] / NP;
            for (int rl = 0; rl < wbnd.nrows[blk]; ++rl) {
                const int r = wbnd.row0[blk] + rl, b = fblk[r];
                for (int cc = clo; cc < chi; ++cc) {
                    if (cc == r) continue;
                    const bool inb = b >= 0 && fblk[cc] == b;
                    if (inb) seen[(size_t)b * 576 + (r - s.qband.row0[b]) * 24 + (cc - s.qband.row0[b])] = 1;
                    for (int p = 0; p < NP; ++p) {
                        const double2 w = wbs[wbnd.off[blk] + ((size_t)(cc - clo) * NP + p) * wbnd.rb + rl];
                        double2 st = make_double2(0, 0);
                        if (inb)
                            st = Ds[((size_t)b * NP + p) * 576 + (r - s.qband.row0[b]) * 24 + (cc - s.qband.row0[b])];
                        md = std::max(md, std::hypot(st.x - w.x, st.y - w.y));
                    }
                }
            }
        }
        for (int b = 0; b < nblk; ++b)
            for (int lr = 0; lr < 24; ++lr)
                for (int lc = 0; lc < 24; ++lc) {
                    if (lr == lc || seen[(size_t)b * 576 + lr * 24 + lc]) continue;
                    for (int p = 0; p < NP; ++p) {
                        const double2 st = Ds[((size_t)b * NP + p) * 576 + lr * 24 + lc];
                        md = std::max(md, std::hypot(st.x, st.y));
                    }
                }
        worst = std::max(worst, md / (rtol * mx));
        dev = std::max(dev, md);
        wmax = std::max(wmax, mx);
    }
    s.mic_check = worst;
    s.mic_dev = dev;
    s.mic_wmax = wmax;
    s.mic_rtol = rtol_max;
    if (worst > 1.0) {
        free_alloc(c, s.Bv);
        free_alloc(c, s.Bs);
        s.Bv = s.Bs = nullptr;
        return;
    }
    std::vector<int> pb, db, pm(nblk, 0);
    for (int b = 0; b < nblk; ++b) {
        bool has = false;
        for (int p : s.pilot_pos) has |= p >= s.qband.row0[b] && p < s.qband.row0[b] + s.qband.nrows[b];
        (has ? pb : db).push_back(b);
        pm[b] = has ? 1 : 0;
    }
    s.npb = (int)pb.size();
    s.ndb = (int)db.size();
    if (s.npb) {
        s.pblk = dupload(c, pb);
        s.pmask = dupload(c, pm);
    }
    if (s.ndb) s.dblk = dupload(c, db);
    build_mic_lr(c, s, a, bv, pb, rinv);
}

// ---------------------------------------------------------------------------
void build_mmse(dsce_ctx* c, Scheme& s, double thr) {
    hipStream_t st = c->stream;
    const int N = s.N, LK = s.LK, NP = s.d.n_pilots, Nsym = s.d.n_tx_symbols, nsnr = c->nsnr;
    std::vector<void*> tmp;
    auto talloc = [&](size_t bytes) {
        void* p;
        DSCE_HIP_CHECK(hipMalloc(&p, bytes));
        tmp.push_back(p);
        return p;
    };
    if (s.W) {                     // rebuild (e.g. new SNR list): back to the structural band
        free_alloc(c, s.W);
        free_alloc(c, s.Wd);
        if (s.Wp3) free_alloc(c, s.Wp3);
        if (s.Wpil) free_alloc(c, s.Wpil);
        if (s.WdA) free_alloc(c, s.WdA);
        if (s.pil_c0) free_alloc(c, s.pil_c0);
        if (s.Bv) free_alloc(c, s.Bv);
        if (s.Bs) free_alloc(c, s.Bs);
        if (s.Bz) free_alloc(c, s.Bz);
        if (s.Tw) free_alloc(c, s.Tw);
        if (s.Ts) free_alloc(c, s.Ts);
        s.Bz = nullptr;
        s.Tw = s.Ts = nullptr;
        s.lr_resid = s.lr_ratio = -1.0;
        if (s.pblk) free_alloc(c, s.pblk);
        if (s.pmask) free_alloc(c, s.pmask);
        if (s.dblk) free_alloc(c, s.dblk);
        s.Bv = s.Bs = nullptr;
        s.pblk = s.pmask = s.dblk = nullptr;
        s.npb = s.ndb = 0;
        s.W = s.Wd = nullptr;
        s.Wp3 = nullptr;
        s.Wpil = s.WdA = nullptr;
        s.pil_c0 = nullptr;
        s.wband = s.wband_struct;
        s.w_elems = s.wband.elems;
        s.Wb = upload_band(c, s.wband, false);
    }
    try {
        double2* dG = (double2*)talloc(s.G.size() * sizeof(double2));
        double2* dQ = (double2*)talloc(s.Q.size() * sizeof(double2));
        double2* dP = (double2*)talloc(s.P.size() * sizeof(double2));
        DSCE_HIP_CHECK(hipMemcpy(dG, s.G.data(), s.G.size() * sizeof(double2), hipMemcpyHostToDevice));
        DSCE_HIP_CHECK(hipMemcpy(dQ, s.Q.data(), s.Q.size() * sizeof(double2), hipMemcpyHostToDevice));
        DSCE_HIP_CHECK(hipMemcpy(dP, s.P.data(), s.P.size() * sizeof(double2), hipMemcpyHostToDevice));
        int* dpil = (int*)talloc(NP * sizeof(int));
        DSCE_HIP_CHECK(hipMemcpy(dpil, s.pilot_pos.data(), NP * sizeof(int), hipMemcpyHostToDevice));
        double* j0tab = (double*)talloc((2 * N - 1) * sizeof(double));
        if (c->ch.model >= 2 && c->ch.fD > 0)     // FastFading.m:331-336: no TimeCorrelation for 'Discrete-*'
            throw ApiError(DSCE_EINVAL, "the time correlation (and so the MMSE estimator) is undefined for a "
                                        "discrete Doppler spectrum (FastFading.m:321-336)");
        setup_time_correlation(st, N, c->ch.fD, c->ch.dt, c->ch.model, j0tab);
        SetupArgs a{};
        a.N = N;
        a.LK = LK;
        a.NP = NP;
        a.Nsym = Nsym;
        a.ntap = c->ch.ntap;
        a.nsnr = nsnr;
        a.pilot_pos = dpil;
        a.G = dG;
        a.Q = dQ;
        a.P = dP;
        a.j0tab = j0tab;
        for (int q = 0; q < c->ch.ntap; ++q) {
            a.tap_delay[q] = c->ch.tap_delay[q];
            a.pdp[q] = c->pdp_norm[c->ch.tap_delay[q]];
        }
        a.kappa = s.d.kappa;
        a.thr = thr;
        double2* m = (double2*)talloc((size_t)NP * a.ntap * N * sizeof(double2));
        setup_mcoef(st, a, s.k.g_start, s.GL, s.k.q_start, s.QL, m);
        double2* rhp = (double2*)talloc((size_t)NP * NP * sizeof(double2));
        setup_rhp(st, a, m, rhp);
        double2* gp = (double2*)talloc((size_t)N * Nsym * sizeof(double2));
        setup_gp(st, a, gp);
        double* dg = (double*)talloc(NP * sizeof(double));
        setup_rest_diag(st, a, gp, s.k.q_start, s.QL, dg);
        std::vector<double2> hrhp((size_t)NP * NP);
        std::vector<double> hdiag(NP);
        DSCE_HIP_CHECK(hipMemcpyAsync(hrhp.data(), rhp, hrhp.size() * sizeof(double2), hipMemcpyDeviceToHost, st));
        DSCE_HIP_CHECK(hipMemcpyAsync(hdiag.data(), dg, NP * sizeof(double), hipMemcpyDeviceToHost, st));
        DSCE_HIP_CHECK(hipStreamSynchronize(st));
        // R_est / R_noI per SNR (script:238-253): tiny NP x NP assembly on the host
        std::vector<double> qn(NP, 0.0);
        for (int i = 0; i < NP; ++i) {
            const int col = s.pilot_pos[i];
            double acc = 0.0;
            for (int n = 0; n < N; ++n) {
                const double2 q = s.Q[(size_t)col * N + n];
                acc += q.x * q.x + q.y * q.y;
            }
            qn[i] = acc;
        }
        s.R_hP = hrhp;
        s.R_est.assign((size_t)nsnr * NP * NP, make_double2(0, 0));
        s.R_noI.assign((size_t)nsnr * NP * NP, make_double2(0, 0));
        for (int k = 0; k < nsnr; ++k) {
            for (int j = 0; j < NP; ++j)
                for (int i = 0; i < NP; ++i) {
                    const size_t ix = (size_t)j * NP + i;
                    double2 noN = i == j ? make_double2(hdiag[i], 0.0) : hrhp[ix];
                    double2 est = noN;
                    if (i == j) est.x = hdiag[i] + c->pn[k] * qn[i] / s.d.kappa;
                    s.R_est[(size_t)k * NP * NP + ix] = est;
                    // R_est - (R_est_noNoise - R_hP)
                    const double2 diff = c_sub(noN, hrhp[ix]);
                    s.R_noI[(size_t)k * NP * NP + ix] = c_sub(est, diff);
                }
        }
        // inverses: [var][snr]
        double2* dR = (double2*)talloc((size_t)2 * nsnr * NP * NP * sizeof(double2));
        double2* dRi = (double2*)talloc((size_t)2 * nsnr * NP * NP * sizeof(double2));
        DSCE_HIP_CHECK(hipMemcpy(dR, s.R_est.data(), (size_t)nsnr * NP * NP * sizeof(double2), hipMemcpyHostToDevice));
        DSCE_HIP_CHECK(hipMemcpy(dR + (size_t)nsnr * NP * NP, s.R_noI.data(), (size_t)nsnr * NP * NP * sizeof(double2),
                                 hipMemcpyHostToDevice));
        setup_rinv(st, NP, 2 * nsnr, dR, dRi);
        // R_Dij packed, then W / W0 per SNR
        double2* rd = (double2*)talloc((size_t)s.w_elems * sizeof(double2));
        Band Wb = s.Wb;
        setup_rdij(st, a, Wb, m, s.k.g_start, s.GL, s.k.q_start, s.QL, rd);
        s.W = dalloc<double2>(c, (size_t)2 * nsnr * s.w_elems);
        s.Wd = dalloc<double2>(c, (size_t)2 * nsnr * LK * NP);
        for (int var = 0; var < 2; ++var)
            for (int k = 0; k < nsnr; ++k) {
                const size_t vi = (size_t)var * nsnr + k;
                setup_w(st, a, Wb, s.w_elems, rd, dRi + vi * NP * NP, s.W + vi * s.w_elems, s.Wd + vi * LK * NP);
            }
        DSCE_HIP_CHECK(hipStreamSynchronize(st));
        DSCE_HIP_CHECK(hipGetLastError());
        trim_w_band(c, s, tmp);
        build_wpair(c, s);
        build_mic(c, s, a, m, dRi);
    } catch (...) {
        for (void* p : tmp) (void)hipFree(p);
        throw;
    }
    for (void* p : tmp) DSCE_HIP_CHECK(hipFree(p));
    s.mmse_ready = true;
}

// ---------------------------------------------------------------------------
// Monte-Carlo batches
// ---------------------------------------------------------------------------
// SNR points processed together by the receiver kernels (Opts::snr_chunk, default
// all): smaller chunks shrink the per-unit working set of a stage.
int snr_chunk(dsce_ctx* c) {
    int k = c->op.snr_chunk;
    if (k <= 0 || k > c->nsnr) k = c->nsnr;
    return k;
}

void ensure_buffers(dsce_ctx* c, int R) {
    size_t N = 0, LK = 0, NP = 0, ND = 0;
    for (auto& s : c->schemes) {
        N = std::max<size_t>(N, s->N);
        LK = std::max<size_t>(LK, s->LK);
        NP = std::max<size_t>(NP, s->d.n_pilots);
        ND = std::max<size_t>(ND, s->d.n_data);
    }
    bool poly = false;      // polyphase perfect-CSI IC scratch: option on and a scheme with the form
    for (auto& sp : c->schemes) poly = poly || (sp->k.poly_ok && c->op.pic_poly);
    const size_t key[8] = {(size_t)R, N, LK, NP, ND, (size_t)snr_chunk(c), (size_t)c->niter, (size_t)poly};
    if (memcmp(key, c->buf_key, sizeof(key)) == 0) return;
    for (void* p : c->buf_allocs) (void)hipFree(p);
    c->buf_allocs.clear();
    memcpy(c->buf_key, key, sizeof(key));
    const size_t U = (size_t)R * snr_chunk(c);
    McBuffers& b = c->buf;
    auto* L = &c->buf_allocs;
    b.R = R;
    b.nsnr = c->nsnr;
    b.U = (int)U;
    // k_pic_mfma reads whole 32-row tiles of y and h and up to 3 samples past N
    // of the taps through block-based buffer views: pad those allocations (zeroed)
    b.ir = dalloc<double2>(c, (size_t)c->ch.ntap * N * R + 4 * (size_t)R, L);
    // samples k_jakes skips (JakesChunks) stay zero
    DSCE_HIP_CHECK(hipMemsetAsync(b.ir, 0, ((size_t)c->ch.ntap * N * R + 4 * (size_t)R) * sizeof(double2), c->stream));
    b.xp = dalloc<double2>(c, NP * R, L);
    b.sidx = dalloc<uint16_t>(c, ND * R, L);
    b.r0 = dalloc<double2>(c, N * R, L);
    b.h = dalloc<double2>(c, (LK + 32) * R, L);
    b.xs = dalloc<double2>(c, LK * R, L);
    b.ss = dalloc<double2>(c, N * R, L);
    b.y = dalloc<double2>(c, (LK + 32) * U, L);
    b.yest = dalloc<double2>(c, LK * U, L);
    b.yperf = dalloc<double2>(c, LK * U, L);
    b.hp = dalloc<double2>(c, NP * U, L);
    b.hp2 = dalloc<double2>(c, NP * U, L);
    b.hest = dalloc<double2>(c, LK * U, L);
    b.v = dalloc<double2>(c, LK * U, L);
    b.u = dalloc<double2>(c, LK * U, L);
    b.t = dalloc<double2>(c, N * U, L);
    b.e = dalloc<double2>(c, LK * U, L);
    b.e2 = dalloc<double2>(c, LK * U, L);
    b.qe = dalloc<uint16_t>(c, ND * U, L);
    b.qp = dalloc<uint16_t>(c, ND * U, L);
    b.sidr = dalloc<uint16_t>(c, (LK + 32) * R, L);
    // LS pilot estimates of every stage (k_mic_pilot -> k_mic_data)
    b.hpa_stages = c->niter + 1;
    b.hpa = dalloc<double2>(c, (size_t)b.hpa_stages * NP * U, L);
    // Z = Bz hP of every stage (low-rank MMSE IC operator, k_mic_pilot -> k_mic_data)
    b.za = dalloc<double2>(c, (size_t)b.hpa_stages * std::max(1, std::min(c->ch.ntap, 2)) * MIC_NB * U, L);
    // polyphase perfect-CSI IC scratch (V and the window sums)
    b.pv = poly ? dalloc<double2>(c, LK * U, L) : nullptr;
    b.pf = poly ? dalloc<double2>(c, LK * U, L) : nullptr;
    b.pf2 = poly ? dalloc<double2>(c, LK * U, L) : nullptr;
    DSCE_HIP_CHECK(hipMemsetAsync(b.sidr, 0, (LK + 32) * R * sizeof(uint16_t), c->stream));
    DSCE_HIP_CHECK(hipMemsetAsync(b.ir + (size_t)c->ch.ntap * N * R, 0, 4 * (size_t)R * sizeof(double2), c->stream));
    DSCE_HIP_CHECK(hipMemsetAsync(b.h + LK * R, 0, 32 * (size_t)R * sizeof(double2), c->stream));
    DSCE_HIP_CHECK(hipMemsetAsync(b.y + LK * U, 0, 32 * U * sizeof(double2), c->stream));
}

// JakesChunks of the context: the union of every scheme's Q^H sample ranges,
// in chunks of JakesChunks::LEN aligned to each range; kept only if it skips at
// least 10 % of the samples (FBMC's overlapping Q^H blocks cover them all).
void update_jakes_chunks(dsce_ctx* c) {
    if (c->jk.n0) free_alloc(c, const_cast<int*>(c->jk.n0));
    if (c->jk.grp) free_alloc(c, const_cast<int2*>(c->jk.grp));
    c->jk = JakesChunks{};
    c->jk_nsch = c->schemes.size();
    const int N = c->ch.N;
    if (N <= 0 || c->schemes.empty()) return;
    std::vector<char> need(N, 0);
    for (auto& sp : c->schemes)
        for (size_t b = 0; b < sp->qband.row0.size(); ++b)
            for (int n = sp->qband.klo[b]; n < sp->qband.khi[b] && n < N; ++n) need[n] = 1;
    std::vector<int> n0;
    int covered = 0;
    for (int n = 0; n < N;) {
        if (!need[n]) {
            ++n;
            continue;
        }
        int e = n;
        while (e < N && need[e]) ++e;
        for (int a = n; a < e; a += JakesChunks::LEN) n0.push_back(a);
        covered += ((e - n + JakesChunks::LEN - 1) / JakesChunks::LEN) * JakesChunks::LEN;
        n = e;
    }
    if (n0.empty() || covered > 0.9 * N) return;
    c->jk.n0 = dupload(c, n0);
    c->jk.n = (int)n0.size();
    c->jk.n0h = n0;
}

// k_jakes_grp's anchor groups for the channel's theta = 2 pi |fD| dt (radians per
// sample): runs of consecutive chunks with theta (span - 1) / 2 <= JAKES_XMAX, MT
// the fewest Taylor terms (16 / 24 / 28) whose remainder x^(MT+1) / (MT+1)!
// is below 1e-17 at the widest run, LG lanes per anchor by the group count.
// Used only when it at least halves the anchors of k_jakes_mom (one per chunk).
void update_jakes_groups(dsce_ctx* c) {
    JakesChunks& jk = c->jk;
    const double th = 6.283185307179586 * std::fabs(c->ch.fD) * c->ch.dt;
    if (jk.theta == th && jk.nsch_grp == jk.n) return;
    if (jk.grp) free_alloc(c, const_cast<int2*>(jk.grp));
    jk.grp = nullptr;
    jk.ngrp = jk.lg = jk.mt = 0;
    jk.theta = th;
    jk.nsch_grp = jk.n;
    const int L = JakesChunks::LEN;
    const std::vector<int>& n0 = jk.n0h;
    if (n0.empty() || !(th > 0.0) || th * 0.5 * (L - 1) > JAKES_XMAX) return;
    // greedy runs of span <= smax samples (first to last sample of the run)
    auto runs = [&](double smax) {
        std::vector<int2> g;
        for (size_t i = 0; i < n0.size();) {
            size_t j = i + 1;
            while (j < n0.size() && (double)(n0[j] + L - 1 - n0[i]) <= smax) ++j;
            g.push_back(make_int2((int)i, (int)(j - i)));
            i = j;
        }
        return g;
    };
    // the fewest runs within |theta k| <= JAKES_XMAX, then (r06) the smallest span
    // that still needs no more runs: C2's 14 windows split 7 + 7 instead of
    // 11 + 3, so the widest run needs MT 24 instead of 28 terms and the anchor
    // lanes' Horner work is balanced
    const int smax_x = (int)std::min(std::floor(2.0 * JAKES_XMAX / th), 1e9);
    std::vector<int2> g = runs(smax_x);
    {
        int lo = L - 1, hi = smax_x;
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (runs(mid).size() <= g.size()) hi = mid;
            else lo = mid + 1;
        }
        g = runs(hi);
    }
    double xmax = 0.0;
    for (const int2& r : g) xmax = std::max(xmax, th * 0.5 * (n0[r.x + r.y - 1] + L - 1 - n0[r.x]));
    if (2 * g.size() > n0.size()) return;
    int mt = 0;
    for (int m : {16, 24, 28}) {                           // 28 covers x <= 3 (7.7e-18)
        double b = 1.0;                                    // x^(m+1) / (m+1)!
        for (int k = 1; k <= m + 1; ++k) b *= xmax / k;
        if (b <= 1e-17) {
            mt = m;
            break;
        }
    }
    if (!mt) return;
    jk.grp = dupload(c, g);
    jk.ngrp = (int)g.size();
    jk.lg = jk.ngrp <= 2 ? 16 : jk.ngrp <= 4 ? 8 : 4;
    jk.mt = mt;
}

// One traced unit (dsce_trace_unit_ex): realisation lane `lane` of the batch at
// SNR index `snr` of scheme `scheme`.  Quantities that sit in a per-unit buffer
// anyway (y, h, hP, and y_est / y_perf of the unfused paths) are copied from
// it; the rest is written by the kernels that form them through TraceK.
struct Trace {
    int scheme, snr, lane;
    const dsce_trace* out;
    TraceK* dev = nullptr;          // device copy of `k`
    TraceK k{};
};

void copy_col(dsce_ctx* c, double* dst, const double2* src, int rows, int stride, int lane) {
    DSCE_HIP_CHECK(hipMemcpy2DAsync(dst, sizeof(double2), src + lane, (size_t)stride * sizeof(double2),
                                    sizeof(double2), rows, hipMemcpyDeviceToHost, c->stream));
}

int var_of_stage(int stage, int niter) { return (stage == 0 || stage <= niter / 2) ? 0 : 1; }

// Realisations [rep0, rep0 + R) with R a multiple of 64; only the first nvalid
// add to the counters / MSE sums (the rest pad a run's tail to whole waves).
void run_batch(dsce_ctx* c, uint64_t seed, uint64_t rep0, int R, int nvalid, Trace* tr) {
    TraceRange trace_range("dsce batch");
    McBuffers& b = c->buf;
    const Opts& op = c->op;
    if (R % 64 || nvalid < 1 || nvalid > R) throw ApiError(DSCE_EINVAL, "run_batch: bad batch geometry");
    b.R = R;
    b.rvalid = nvalid;
    b.tr = nullptr;
    {
        Timed t(c, "k_jakes");
        if (c->jk_nsch != c->schemes.size()) update_jakes_chunks(c);
        update_jakes_groups(c);
        c->jakes_kind = launch_jakes(c->stream, op, c->ch, seed, rep0, R, b.ir, &c->jk);
    }
    const int chunk = snr_chunk(c);
    for (size_t si = 0; si < c->schemes.size(); ++si) {
        Scheme& s = *c->schemes[si];
        s.path = 0;
        MmseK mm{};
        mm.W = s.W;
        mm.Wd = s.Wd;
        mm.w_elems = s.w_elems;
        mm.nsnr = c->nsnr;
        mm.Wb = s.Wb;
        mm.Wp3 = s.Wp3;
        mm.wp_elems = s.wp_elems;
        mm.Pb = s.Pb;
        mm.Wpil = s.Wpil;
        mm.WdA = s.WdA;
        mm.pil_c0 = s.pil_c0;
        mm.Bv = s.Bv;
        mm.Bs = s.Bs;
        mm.pblk = s.pblk;
        mm.pmask = s.pmask;
        mm.npb = s.npb;
        mm.dblk = s.dblk;
        mm.ndb = s.ndb;
        mm.Bz = s.Bz;
        mm.Tw = s.Tw;
        mm.Ts = s.Ts;
        {
            Timed t(c, "tx");
            b.U = R * std::min(chunk, c->nsnr);
            launch_tx(c->stream, s.k, c->ch, s.d.bits_slot, s.d.pilot_slot, seed, rep0, b,
                      txrx_fft_ok(op, s.k, c->ch, b), op.tx_rows != 0);
        }
        const bool pfuse = perfect_fusable(op, s.k);
        for (int s0 = 0; s0 < c->nsnr; s0 += chunk) {
            b.snr0 = s0;
            b.U = R * std::min(chunk, c->nsnr - s0);
            const bool tracing = tr && tr->scheme == (int)si && tr->snr >= s0 && tr->snr < s0 + chunk;
            const int tunit = tracing ? (tr->snr - s0) * R + tr->lane : 0;
            if (tracing) {
                tr->k.unit = tunit;
                DSCE_HIP_CHECK(hipMemcpyAsync(tr->dev, &tr->k, sizeof(TraceK), hipMemcpyHostToDevice, c->stream));
            }
            b.tr = tracing ? tr->dev : nullptr;
            const dsce_trace* to = tracing ? tr->out : nullptr;
            const int LK = s.LK, NP = s.d.n_pilots;
            {
                Timed t(c, "rx_front");
                s.path |= launch_rx_front(c->stream, op, s.k, c->ch, c->d_pn, seed, rep0, b);
            }
            if (to && to->y) copy_col(c, to->y, b.y, LK, b.U, tunit);
            if (to && to->h_perfect) copy_col(c, to->h_perfect, b.h, LK, R, tr->lane);
            // FFT-form OFDM: the perfect-CSI branch is one k_pic_fft with its
            // stage 0, the MMSE branch k_mic_pilot + k_mic_data, every stage each
            if (pfuse && mmse_stages_ok(op, s.k, mm, c->ch, b, c->niter)) {
                PerfectDetectArgs pd{c->d_counters, (int)si, 0, c->niter + 1, c->nsnr, 0, s.k.slI, s.k.slQ};
                // the low-rank tap operator (both passes or neither: the data pass
                // reads the pilot pass's Z instead of its LS pilots)
                const bool lr = op.mic_lr && (op.mic_net & 1) && s.Bz;
                // (r06: the r05 options ic_streams 2 / 3 — the chain on a second
                // stream, or beside the pilot pass in one launch, k_ic_pair — were
                // within box noise and are retired; "ic_stages" spans the group)
                {
                    Timed tg(c, "ic_stages");
                    {
                        Timed t(c, "perfect_ic");
                        s.path |= launch_perfect_chain(c->stream, op, s.k, c->ch, b, &pd, c->niter, true);
                    }
                    {
                        Timed t(c, "k_mic_pilot");
                        s.path |= launch_mmse_stages(c->stream, s.k, mm, c->ch, b, &pd, c->niter, op.xcd, 1,
                                                     (op.mic_net & 2) != 0, lr);
                    }
                    {
                        Timed t(c, "k_mic_data");
                        s.path |= launch_mmse_stages(c->stream, s.k, mm, c->ch, b, &pd, c->niter, op.xcd, 2,
                                                     (op.mic_net & 1) != 0, lr);
                    }
                }
                if (to && to->hp_stages)
                    for (int st = 0; st <= c->niter; ++st)
                        copy_col(c, to->hp_stages + (size_t)2 * st * NP, b.hpa + (size_t)st * NP * b.U, NP, b.U, tunit);
                b.tr = nullptr;
                continue;
            }
            // Otherwise one launch group per stage.  With the perfect-CSI branch
            // fused into perfect_ic, the IC iterations are two independent chains
            // after stage 0: MMSE (contraction -> stage) and perfect CSI.
            // FFT-form OFDM with the W contraction (mmse_ic 0): the whole
            // perfect-CSI chain is one kernel (k_pic_fft, u in registers)
            const bool chain = pfuse && perfect_chain_ok(op, s.k, c->ch, b, c->niter);
            // block-diagonal W + row-local P (OFDM): the MMSE stage of every IC
            // iteration rides in the contraction's epilogue (k_pilot_pre +
            // k_wpair3<..., true>); hP alternates between hp and hp2
            const bool mfuse = pfuse && mmse_fused_ok(op, s.k, mm, b);
            double2* hp_prev = b.hp;
            double2* hp_cur = b.hp2;
            for (int it = 0; it <= c->niter; ++it) {
                if (it == 1 && chain) {
                    Timed t(c, "perfect_ic");
                    PerfectDetectArgs pd{c->d_counters, (int)si, 1, c->niter + 1, c->nsnr, 0, s.k.slI, s.k.slQ};
                    s.path |= launch_perfect_chain(c->stream, op, s.k, c->ch, b, &pd, c->niter);
                }
                if (it > 0 && mfuse) {
                    {
                        Timed t(c, "k_pilot_pre");
                        launch_pilot_pre(c->stream, s.k, mm, var_of_stage(it - 1, c->niter), b, hp_prev, hp_cur);
                    }
                    if (to && to->hp_stages) copy_col(c, to->hp_stages + (size_t)2 * it * NP, hp_cur, NP, b.U, tunit);
                    {
                        // the contraction with the stage in its epilogue
                        Timed t(c, "k_wcontract");
                        s.path |= launch_mmse_fused(c->stream, op, s.k, mm, var_of_stage(it - 1, c->niter),
                                                    var_of_stage(it, c->niter), it, c->niter, it == c->niter, b,
                                                    hp_prev, hp_cur, c->d_counters, (int)si);
                    }
                    std::swap(hp_prev, hp_cur);
                    if (!chain) {
                        Timed t(c, "perfect_ic");
                        PerfectDetectArgs pd{c->d_counters, (int)si, it, c->niter + 1, c->nsnr, it == c->niter,
                                             s.k.slI, s.k.slQ};
                        s.path |= launch_perfect_ic(c->stream, op, s.k, c->ch, b, pfuse ? &pd : nullptr);
                    }
                    continue;
                }
                if (it > 0) {
                    {
                        Timed t(c, "k_wcontract");
                        s.path |= launch_wcontract(c->stream, op, s.k, mm, var_of_stage(it - 1, c->niter), b);
                    }
                    if (to && to->yest_stages) copy_col(c, to->yest_stages + (size_t)2 * it * LK, b.yest, LK, b.U, tunit);
                    if (!chain) {
                        Timed t(c, "perfect_ic");
                        PerfectDetectArgs pd{c->d_counters, (int)si, it, c->niter + 1, c->nsnr, it == c->niter,
                                             s.k.slI, s.k.slQ};
                        s.path |= launch_perfect_ic(c->stream, op, s.k, c->ch, b, pfuse ? &pd : nullptr);
                        if (to && to->yperf_stages && !pfuse)
                            copy_col(c, to->yperf_stages + (size_t)2 * it * LK, b.yperf, LK, b.U, tunit);
                    }
                }
                {
                    Timed t(c, "k_stage");
                    s.path |= launch_stage(c->stream, op, s.k, mm, it, var_of_stage(it, c->niter), c->niter,
                                           it == c->niter, b, c->d_counters, (int)si, !(pfuse && it > 0));
                }
                if (to && to->hp_stages) copy_col(c, to->hp_stages + (size_t)2 * it * NP, b.hp, NP, b.U, tunit);
            }
            b.tr = nullptr;
        }
    }
    DSCE_HIP_CHECK(hipGetLastError());
}

// Noise sub-streams (include/dsce.h NOISE): SNR index k of noise slot g draws
// sub-stream snr_base + k + 256 g, a 16-bit field.  With any slot > 0 the SNR
// part must stay below 256 or the streams of slot g would run into slot g + 1's.
void check_noise_streams(const dsce_ctx* c, long long base, long long nsnr, int max_slot) {
    if (max_slot > 0 && base + nsnr > 256)
        throw ApiError(DSCE_EINVAL, "snr_base + n_snr must be <= 256 when a scheme uses noise slot > 0 (got " +
                                        std::to_string(base) + " + " + std::to_string(nsnr) + ")");
    if (base + nsnr + 256LL * max_slot > 65536) throw ApiError(DSCE_EINVAL, "noise sub-stream index exceeds 16 bits");
}

int max_noise_slot(const dsce_ctx* c) {
    int m = 0;
    for (auto& s : c->schemes) m = std::max(m, s->k.noise_slot);
    return m;
}

int api_fail(dsce_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

// API_END: every entry point that launched work returns the launch errors it
// left (check_ctx clears stale errors at entry, so an error not
// checked before returning would otherwise be lost)
#define API_BEGIN try {
#define API_END                                                 \
    DSCE_HIP_CHECK(hipGetLastError());                          \
    }                                                           \
    catch (const ApiError& e) { return api_fail(ctx, e.code, e.what()); } \
    catch (const HipError& e) { return api_fail(ctx, DSCE_EHIP, e.what()); } \
    catch (const std::bad_alloc&) { return api_fail(ctx, DSCE_ENOMEM, "host out of memory"); } \
    catch (const std::exception& e) { return api_fail(ctx, DSCE_EINVAL, e.what()); }     \
    return DSCE_OK;

// Algorithmic work per realisation of one timed kernel group of a scheme
// (dsce_kernel_work).  Flops: 8 per complex multiply-accumulate, 2 per real
// FMA, 5 n log2 n per n-point DFT (the FFT convention), transcendental
// functions (cis, log, sqrt) and the RNG's integer work not counted.  Bytes:
// the compulsory HBM traffic, every operand read once per realisation or unit
// and every result written once (L2 reuse across the SNR points assumed).
// Only the kernel groups whose form is fixed by the path are modelled: the
// FFT-form OFDM chain of C2 (k_jakes_grp / k_jakes_mom, k_tx_rows, k_txrx_fft,
// k_pic_fft, k_mic_pilot, k_mic_data) and the W contraction; other groups
// return 0 (unmodelled).
struct KWork {
    double flops = 0.0, bytes = 0.0;
};

KWork kernel_work(const dsce_ctx* c, const Scheme& s, const std::string& name) {
    KWork w;
    if (name == "ic_stages") {
        // the IC group of the FFT-form OFDM path: k_pic_fft, k_mic_pilot, k_mic_data
        if (!(s.path & PATH_MIC_STAGES)) return w;
        for (const char* g : {"perfect_ic", "k_mic_pilot", "k_mic_data"}) {
            const KWork x = kernel_work(c, s, g);
            w.flops += x.flops;
            w.bytes += x.bytes;
        }
        return w;
    }
    const double nt = c->ch.ntap, NP = s.d.n_pilots, ns = c->nsnr, it = c->niter, LK = s.LK;
    const double DFT = 5.0 * 24.0 * std::log2(24.0);
    const bool fft = (s.path & PATH_MIC_STAGES) != 0;
    const double nblk = s.k.QH.nblk, B16 = sizeof(double2);
    if (name == "k_jakes") {
        // per non-zero tap and read sample window: the path moments of each
        // anchor (MT terms x (real scale + complex add) per path) and the
        // Horner evaluation per sample (MT x one complex multiply-add by j k)
        const double nch = c->jk.n, P = c->ch.paths;
        double mt = 0.0, anchors = 0.0;
        if (c->jakes_kind == JAKES_KIND_GRP) {
            mt = c->jk.mt;
            anchors = c->jk.ngrp;
        } else if (c->jakes_kind == JAKES_KIND_MOM) {
            mt = 12;
            anchors = nch;
        }
        if (mt > 0) {
            w.flops = nt * 4.0 * mt * (anchors * P + nch * JakesChunks::LEN);
            w.bytes = nt * nch * JakesChunks::LEN * B16;
        }
        return w;
    }
    if (name == "k_wcontract" && !fft) {
        const double fused = (s.path & PATH_WPAIR3_FUSED) ? LK * NP : 0.0;
        w.flops = 8.0 * ((double)(s.w_struct - s.w_diag) + fused) * ns * it;
        // per unit and iteration: y, hP and v read, y_est written (W itself is
        // shared by the batch: dsce_work_model's bytes per SNR point)
        w.bytes = ns * it * (3.0 * LK + NP) * B16;
        return w;
    }
    if (name == "perfect_ic" && (s.path & PATH_PIC_POLY)) {
        // polyphase passes per unit and IC iteration: C u and an IDFT-F per
        // symbol, the synthesis window sums (nnz(A) real x complex MACs per tap),
        // the channel (nt CMACs per sample), the analysis window sums (nnz(B)),
        // a DFT-F and E per symbol, y - out + h u per row; bytes: u, y, h read
        // and y_perf written (V and the window sums are the kernels' own scratch)
        const double F = s.k.poly_F, K = s.k.poly_K, DF = 5.0 * F * std::log2(F);
        const double per = 2.0 * K * (DF + 8.0 * F) + 4.0 * nt * s.poly_nnz_a + 8.0 * nt * s.N +
                           4.0 * s.poly_nnz_b + 16.0 * LK;
        w.flops = ns * it * per;
        w.bytes = ns * it * 3.0 * LK * B16 + it * LK * B16;
        return w;
    }
    if (!fft) return w;
    const double npb = s.npb, ndb = s.ndb;
    // one IC stage of one symbol and unit, both estimators: IDFT24 of the
    // decisions, the channel (nt x 24 CMACs), DFT24, y_ic / one-tap per row
    // (residual + diag(D_hat) v: 2 CMACs, quotient: 1 complex division = 2
    // CMACs), re-precoding (1 CMAC)
    const double chain = 2.0 * DFT + 8.0 * (nt * 24.0 + 24.0 * 5.0);
    // the MMSE extras per stage and symbol: the estimated taps (nt x 24 x NP
    // complex MACs; low-rank operator: nt x 24 x MIC_NB real x complex MACs at 4
    // flops), this stage's window sums (Bs hP: nt x NP; low-rank: nt x MIC_NB real
    // x complex), diag(D_hat) per row (nt CMACs)
    const bool lrp = (s.path & PATH_MIC_LR) != 0;
    const double mmse_extra = lrp ? 4.0 * (nt * 24.0 * MIC_NB + nt * MIC_NB) + 8.0 * nt * 24.0
                                  : 8.0 * (nt * 24.0 * NP + nt * NP + nt * 24.0);
    const double stage0 = 8.0 * (24.0 * 3.0);             // one-tap quotient + re-precoding per row
    if (name == "tx") {
        w.flops = 8.0 * LK;                                // P [xP; xD] (row-local precoder: 1 CMAC per row)
        w.bytes = LK * (B16 + sizeof(uint16_t)) + NP * B16 + s.d.n_data * sizeof(uint16_t);
    } else if (name == "rx_front") {
        // per symbol: s = gs IDFT24(x), r0 = H s, diag(D) (window sums + one CMAC
        // per row); per SNR point: r0 + sqrt(Pn/2) z (2 FMAs per sample), y = qs DFT24(r)
        w.flops = nblk * (DFT + 8.0 * nt * 24.0 + 2.0 * nt * 24.0 + 8.0 * 24.0 + ns * (4.0 * 24.0 + DFT));
        w.bytes = (LK + nt * nblk * 24.0 + LK + ns * LK) * B16;
    } else if (name == "perfect_ic") {
        // per unit and symbol: stage 0 one-tap, then it IC iterations of the chain
        w.flops = ns * nblk * (stage0 + it * chain);
        w.bytes = (ns * LK + 2.0 * LK + nt * nblk * 24.0) * B16 + LK * sizeof(uint16_t);
    } else if (name == "k_mic_pilot" || name == "k_mic_data") {
        const double nsym = name == "k_mic_pilot" ? npb : ndb;
        // stage 0: LS / window sums + one-tap; stages 1..it: chain + MMSE extras
        w.flops = ns * nsym * (stage0 + (lrp ? 4.0 * nt * MIC_NB : 8.0 * nt * NP) + it * (chain + mmse_extra));
        if (name == "k_mic_pilot") {
            w.flops += ns * (it + 1) * NP * 8.0;                          // LS: y_P / x_P / sqrt(kappa)
            if (lrp) w.flops += ns * (it + 1) * nt * MIC_NB * NP * 8.0;   // Z = Bz hP, once per unit and stage
        }
        const double ysym = ns * nsym * 24.0 * B16;                       // y of the kernel's symbols
        // hP of every stage written (pilot) or read (data); low-rank: Z instead
        const double hpa = ns * (it + 1) * (lrp ? nt * MIC_NB : NP) * B16;
        w.bytes = ysym + hpa + nsym * 24.0 * (B16 + sizeof(uint16_t));    // + xs, sidr of the symbols
    }
    return w;
}

}  // namespace

// ---- multi-device contexts (dsce_create_multi, ABI 7) -----------------------
#define DSCE_NCCL_CHECK(x)                                                                             \
    do {                                                                                               \
        const ncclResult_t r_ = (x);                                                                   \
        if (r_ != ncclSuccess)                                                                         \
            throw ApiError(DSCE_EHIP, std::string("RCCL error '") + ncclGetErrorString(r_) + "' (" #x ")"); \
    } while (0)

static dsce_ctx* member(dsce_ctx* ctx, size_t m) { return m ? ctx->peers[m - 1] : ctx; }

static std::string member_name(const dsce_ctx* ctx, size_t m) {
    const dsce_ctx* c = m ? ctx->peers[m - 1] : ctx;
    return "member " + std::to_string(m) + " (device " + std::to_string(c->device) + ")";
}

// A configuration call on a multi-device context runs on every member, member 0
// first (it validates the arguments; the members are configured identically,
// so a later member fails only on its own device's resources).
template <class F>
static int fanout(dsce_ctx* ctx, F&& f) {
    const int rc = f(ctx);
    if (rc != DSCE_OK || !ctx) return rc;
    for (size_t m = 1; m <= ctx->peers.size(); ++m) {
        const int r2 = f(member(ctx, m));
        if (r2 != DSCE_OK) return api_fail(ctx, r2, member_name(ctx, m) + ": " + member(ctx, m)->err);
    }
    return DSCE_OK;
}

// The same with one host thread per member (dsce_build_mmse: the setup is
// replicated per device, SURVEY §8e, and runs concurrently).
template <class F>
static int fanout_par(dsce_ctx* ctx, F&& f) {
    if (!ctx || ctx->peers.empty()) return f(ctx);
    const size_t n = ctx->peers.size() + 1;
    std::vector<int> rc(n, DSCE_OK);
    std::vector<std::thread> th;
    try {
        for (size_t m = 1; m < n; ++m) th.emplace_back([&, m] { rc[m] = f(member(ctx, m)); });
    } catch (const std::exception& e) {
        for (auto& t : th) t.join();
        return api_fail(ctx, DSCE_ENOMEM, std::string("cannot start a member thread: ") + e.what());
    }
    rc[0] = f(ctx);
    for (auto& t : th) t.join();
    if (rc[0] != DSCE_OK) return rc[0];
    for (size_t m = 1; m < n; ++m)
        if (rc[m] != DSCE_OK) return api_fail(ctx, rc[m], member_name(ctx, m) + ": " + member(ctx, m)->err);
    return DSCE_OK;
}

// Slice m of [first, first + n) over `world` members on multiples of 64
// realisations (dsce/parallel.py shard_range, the torch.distributed twin)
static void shard_slice(uint64_t first, uint64_t n, size_t world, size_t m, uint64_t& f, uint64_t& k) {
    const uint64_t blocks = (n + 63) / 64;
    const uint64_t lo = std::min<uint64_t>(blocks * m / world * 64, n);
    const uint64_t hi = std::min<uint64_t>(blocks * (m + 1) / world * 64, n);
    f = first + lo;
    k = hi - lo;
}

extern "C" {

int dsce_abi_version(void) { return DSCE_ABI_VERSION; }

int dsce_device_count(int* count) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (count) *count = n;
    return DSCE_OK;
}

int dsce_create(int hip_device, dsce_ctx** out) {
    if (!out) return DSCE_EINVAL;
    *out = nullptr;
    auto* ctx = new (std::nothrow) dsce_ctx();
    if (!ctx) return DSCE_ENOMEM;
    ctx->device = hip_device;
    try {
        DSCE_HIP_CHECK(hipSetDevice(hip_device));
        DSCE_HIP_CHECK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    } catch (const std::exception& e) {
        delete ctx;
        return DSCE_EHIP;
    }
    *out = ctx;
    return DSCE_OK;
}

int dsce_create_multi(const int32_t* devices, int32_t n_devices, dsce_ctx** out) {
    if (!out) return DSCE_EINVAL;
    *out = nullptr;
    if (!devices || n_devices < 1 || n_devices > 64) {
        fprintf(stderr, "dsce_create_multi: 1..64 devices expected\n");
        return DSCE_EINVAL;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    bool distinct = true;
    for (int i = 0; i < n_devices; ++i) {
        if (devices[i] < 0 || devices[i] >= count) {
            fprintf(stderr, "dsce_create_multi: device %d of %d is not a HIP device\n", (int)devices[i], count);
            return DSCE_EINVAL;
        }
        for (int j = 0; j < i; ++j) distinct = distinct && devices[j] != devices[i];
    }
    dsce_ctx* ctx = nullptr;
    int rc = dsce_create(devices[0], &ctx);
    if (rc != DSCE_OK) return rc;
    for (int i = 1; i < n_devices; ++i) {
        dsce_ctx* p = nullptr;
        rc = dsce_create(devices[i], &p);
        if (rc != DSCE_OK) {
            (void)dsce_destroy(ctx);
            return rc;
        }
        ctx->peers.push_back(p);
    }
    if (distinct) {
        // one communicator per member in this process (single-process multi-GPU
        // RCCL); n_devices = 1 too, so the reduction path is the same at any size
        ctx->comms.assign(n_devices, nullptr);
        const ncclResult_t r = ncclCommInitAll(ctx->comms.data(), n_devices, devices);
        if (r != ncclSuccess) {
            fprintf(stderr, "dsce_create_multi: ncclCommInitAll failed: %s\n", ncclGetErrorString(r));
            ctx->comms.clear();
            (void)dsce_destroy(ctx);
            return DSCE_EHIP;
        }
        ctx->reduce = DSCE_REDUCE_RCCL;
    } else {
        ctx->reduce = DSCE_REDUCE_HOST;
    }
    (void)hipSetDevice(devices[0]);
    *out = ctx;
    return DSCE_OK;
}

int dsce_group_info(dsce_ctx* ctx, int32_t* n_devices, int32_t* devices, int32_t* reduce) {
    if (!ctx) return DSCE_EINVAL;
    const size_t n = ctx->peers.size() + 1;
    if (n_devices) *n_devices = (int32_t)n;
    if (devices)
        for (size_t m = 0; m < n; ++m) devices[m] = member(ctx, m)->device;
    if (reduce) *reduce = ctx->reduce;
    return DSCE_OK;
}

int dsce_destroy(dsce_ctx* ctx) {
    if (!ctx) return DSCE_OK;
    // a multi-device handle: its communicators, then its members (each reports
    // its own failing call on stderr)
    int member_rc = DSCE_OK;
    for (ncclComm_t cm : ctx->comms)
        if (cm && ncclCommDestroy(cm) != ncclSuccess) {
            fprintf(stderr, "dsce_destroy: ncclCommDestroy failed\n");
            member_rc = DSCE_EHIP;
        }
    ctx->comms.clear();
    for (dsce_ctx* p : ctx->peers)
        if (dsce_destroy(p) != DSCE_OK) member_rc = DSCE_EHIP;
    ctx->peers.clear();
    // The context is freed whatever happens; a failing call is named (stderr),
    // its error cleared, so it does not surface in the next context's
    // hipGetLastError (r04: a stale 'invalid argument' met a later build_mmse),
    // and returned as DSCE_EHIP (ABI 6: the r04 double free was only printed).
    const char* first = nullptr;
    hipError_t ferr = hipSuccess;
    auto note = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && !first) {
            first = what;
            ferr = e;
        }
    };
    note(hipSetDevice(ctx->device), "hipSetDevice");
    if (ctx->stream) note(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    for (void* p : ctx->buf_allocs) note(hipFree(p), "hipFree (batch buffers)");
    for (void* p : ctx->allocs) note(hipFree(p), "hipFree (operators)");
    if (ctx->h_counters) note(hipHostFree(ctx->h_counters), "hipHostFree (counters)");
    for (auto& e : ctx->pending) {
        note(hipEventDestroy(e.a), "hipEventDestroy");
        note(hipEventDestroy(e.b), "hipEventDestroy");
    }
    for (auto e : ctx->event_pool) note(hipEventDestroy(e), "hipEventDestroy (pool)");
    if (ctx->stream) note(hipStreamDestroy(ctx->stream), "hipStreamDestroy");
    delete ctx;
    if (first) fprintf(stderr, "dsce_destroy: %s failed: %s\n", first, hipGetErrorString(ferr));
    (void)hipGetLastError();
    return first ? DSCE_EHIP : member_rc;
}

const char* dsce_last_error(const dsce_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static int set_channel_one(dsce_ctx* ctx, const dsce_channel_desc* d) {
    TraceRange trace_range("dsce_set_channel");
    API_BEGIN
    check_ctx(ctx);
    if (!d || !d->pdp_norm || d->n_samples <= 1 || d->n_taps <= 0 || d->n_paths <= 0 || d->sampling_rate <= 0)
        throw ApiError(DSCE_EINVAL, "invalid channel description");
    if (d->doppler_model < 0 || d->doppler_model > 3) throw ApiError(DSCE_EINVAL, "doppler_model must be 0..3");
    if (!ctx->schemes.empty()) throw ApiError(DSCE_ESTATE, "set the channel before adding schemes");
    ChannelK ch{};
    ch.N = d->n_samples;
    ch.fD = d->max_doppler;
    ch.dt = 1.0 / d->sampling_rate;
    ch.paths = d->n_paths;
    ch.model = d->doppler_model;
    ctx->pdp_norm.assign(d->pdp_norm, d->pdp_norm + d->n_taps);
    int nt = 0;
    for (int i = 0; i < d->n_taps; ++i) {
        if (d->pdp_norm[i] != 0.0) {
            if (nt >= 8) throw ApiError(DSCE_EINVAL, "at most 8 non-zero channel taps are supported");
            ch.tap_delay[nt] = i;
            ch.sqrt_pdp[nt] = sqrt(d->pdp_norm[i]);
            ++nt;
        }
    }
    if (nt == 0) throw ApiError(DSCE_EINVAL, "power delay profile is all zero");
    if (!(d->max_doppler >= 0)) throw ApiError(DSCE_EINVAL, "max_doppler must be >= 0");
    ch.ntap = nt;
    if (ch.model >= 2 && ch.fD > 0) {
        // discrete Doppler spectrum, FastFading.m:153-177
        const double df = d->sampling_rate / d->n_samples;
        if (ch.fD / df <= 0.5) {
            ch.fD = 0.0;                                   // FastFading.m:153-156: velocity set to zero
        } else {
            const int nd = (int)ceil(ch.fD / df);
            if (2 * nd + 1 > d->n_samples) throw ApiError(DSCE_EINVAL, "discrete Doppler spectrum wider than N");
            std::vector<double> ip(2 * nd + 2), spec(2 * nd + 1);
            for (int i = 0; i < 2 * nd + 2; ++i) {
                double v = df * ((double)(i - nd - 1) + 0.5);
                if (v <= -ch.fD) v = -ch.fD;
                if (v >= ch.fD) v = ch.fD;
                ip[i] = v;
            }
            double sum = 0.0;
            for (int i = 0; i < 2 * nd + 1; ++i) {
                spec[i] = ch.model == 2 ? asin(ip[i + 1] / ch.fD) - asin(ip[i] / ch.fD) : ip[i + 1] - ip[i];
                sum += spec[i];
            }
            for (auto& v : spec) v = sqrt(v / sum);
            ch.nd = nd;
            ch.sqrt_dspec = dupload(ctx, spec);
        }
    }
    ctx->ch = ch;
    ctx->chan_set = true;
    API_END
}

int dsce_set_channel(dsce_ctx* ctx, const dsce_channel_desc* d) {
    return fanout(ctx, [&](dsce_ctx* c) { return set_channel_one(c, d); });
}

static int set_snr_one(dsce_ctx* ctx, const double* pn_time, int32_t n_snr, int32_t n_iter) {
    API_BEGIN
    check_ctx(ctx);
    if (!pn_time || n_snr <= 0 || n_iter < 0) throw ApiError(DSCE_EINVAL, "invalid SNR list");
    check_noise_streams(ctx, ctx->op.snr_base, n_snr, max_noise_slot(ctx));
    ctx->pn.assign(pn_time, pn_time + n_snr);
    ctx->nsnr = n_snr;
    ctx->niter = n_iter;
    if (ctx->d_pn) free_alloc(ctx, ctx->d_pn);
    ctx->d_pn = dupload(ctx, ctx->pn);
    for (auto& s : ctx->schemes) {
        s->mmse_ready = false;
        if (s->interp) upload_interp(ctx, *s);
    }
    const size_t n = ctx->schemes.size() * 4 * (size_t)n_snr * (n_iter + 1);
    ctx->counters_n = 0;
    (void)n;
    API_END
}

int dsce_set_snr(dsce_ctx* ctx, const double* pn_time, int32_t n_snr, int32_t n_iter) {
    return fanout(ctx, [&](dsce_ctx* c) { return set_snr_one(c, pn_time, n_snr, n_iter); });
}

static int add_scheme_one(dsce_ctx* ctx, const dsce_scheme_desc* d, int32_t* scheme_id) {
    TraceRange trace_range("dsce_add_scheme");
    API_BEGIN
    check_ctx(ctx);
    if (!ctx->chan_set) throw ApiError(DSCE_ESTATE, "dsce_set_channel first");
    if (!d || !d->G || !d->Q || !d->P || !d->pilot_pos || !d->considered || !d->symbols)
        throw ApiError(DSCE_EINVAL, "null operator");
    const int LK = d->n_subcarriers * d->n_symbols;
    if (LK <= 0 || d->n_pilots <= 0 || d->n_pilots > DSCE_MAX_NP || d->n_data <= 0 ||
        d->n_tx_symbols != d->n_pilots + d->n_data)
        throw ApiError(DSCE_EINVAL, "inconsistent scheme dimensions");
    if (d->mod_order < 2 || d->mod_order > 256 || (d->mod_order & (d->mod_order - 1)) ||
        (1 << d->bits_per_symbol) != d->mod_order || 32 % d->bits_per_symbol)
        throw ApiError(DSCE_EINVAL, "modulation order must be a power of two <= 256");
    if (!d->despread && !d->data_pos) throw ApiError(DSCE_EINVAL, "data_pos required in select mode");
    if (d->kappa <= 0 || d->data_div <= 0) throw ApiError(DSCE_EINVAL, "kappa/data_div must be positive");
    auto s = std::make_unique<Scheme>();
    s->d = *d;
    s->N = ctx->ch.N;
    s->LK = LK;
    const size_t nG = (size_t)s->N * LK;
    s->G.resize(nG);
    s->Q.resize(nG);
    for (size_t i = 0; i < nG; ++i) {
        s->G[i] = cx(d->G, i);
        s->Q[i] = cx(d->Q, i);
    }
    s->P.resize((size_t)LK * d->n_tx_symbols);
    for (size_t i = 0; i < s->P.size(); ++i) s->P[i] = cx(d->P, i);
    s->pilot_pos.assign(d->pilot_pos, d->pilot_pos + d->n_pilots);
    for (int p : s->pilot_pos)
        if (p < 0 || p >= LK) throw ApiError(DSCE_EINVAL, "pilot position out of range");
    if (!d->despread) {
        s->data_pos.assign(d->data_pos, d->data_pos + d->n_data);
        for (int p : s->data_pos)
            if (p < 0 || p >= LK) throw ApiError(DSCE_EINVAL, "data position out of range");
    } else {
        s->data_pos.assign(1, 0);
    }
    s->considered.assign(d->considered, d->considered + d->n_data);
    s->symbols.resize(d->mod_order);
    for (int m = 0; m < d->mod_order; ++m) s->symbols[m] = cx(d->symbols, m);
    pack_scheme(ctx, *s);
    if (scheme_id) *scheme_id = (int32_t)ctx->schemes.size();
    ctx->schemes.push_back(std::move(s));
    API_END
}

int dsce_add_scheme(dsce_ctx* ctx, const dsce_scheme_desc* d, int32_t* scheme_id) {
    return fanout(ctx, [&](dsce_ctx* c) { return add_scheme_one(c, d, scheme_id); });
}

static int build_mmse_one(dsce_ctx* ctx, double zero_threshold) {
    TraceRange trace_range("dsce_build_mmse");
    API_BEGIN
    check_ctx(ctx);
    if (ctx->nsnr <= 0) throw ApiError(DSCE_ESTATE, "dsce_set_snr first");
    if (ctx->schemes.empty()) throw ApiError(DSCE_ESTATE, "no scheme added");
    for (auto& s : ctx->schemes)
        if (!s->interp) build_mmse(ctx, *s, zero_threshold);
    API_END
}

int dsce_build_mmse(dsce_ctx* ctx, double zero_threshold) {
    return fanout_par(ctx, [&](dsce_ctx* c) { return build_mmse_one(c, zero_threshold); });
}

static int set_batch_one(dsce_ctx* ctx, int32_t reps) {
    API_BEGIN
    check_ctx(ctx);
    if (reps < 64) throw ApiError(DSCE_EINVAL, "batch must be >= 64");
    ctx->batch = (reps + 63) / 64 * 64;
    API_END
}

int dsce_set_batch(dsce_ctx* ctx, int32_t reps) {
    return fanout(ctx, [&](dsce_ctx* c) { return set_batch_one(c, reps); });
}

static void prepare_run(dsce_ctx* ctx) {
    if (ctx->schemes.empty()) throw ApiError(DSCE_ESTATE, "no scheme added");
    for (auto& s : ctx->schemes) {
        if (!s->mmse_ready) throw ApiError(DSCE_ESTATE, "dsce_build_mmse first");
        if (s->interp && ctx->niter > 0)
            throw ApiError(DSCE_ESTATE, "interference-cancellation iterations need the MMSE estimator (n_iter must be 0 "
                                        "with an interpolation estimator)");
    }
    const size_t n = ctx->schemes.size() * 4 * (size_t)ctx->nsnr * (ctx->niter + 1);
    if (ctx->counters_n != n) {
        ctx->d_counters = dalloc<unsigned long long>(ctx, n);
        ctx->counters_n = n;
    }
    DSCE_HIP_CHECK(hipMemsetAsync(ctx->d_counters, 0, n * sizeof(unsigned long long), ctx->stream));
    ctx->buf.mse_err = ctx->buf.mse_pow = nullptr;
    if (ctx->mse) {
        const size_t ns = ctx->schemes.size(), ne = ns * ctx->nsnr * (ctx->niter + 1), np = ns * ctx->nsnr;
        if (ctx->mse_n != ne + np) {
            if (ctx->d_mse) free_alloc(ctx, ctx->d_mse);
            ctx->d_mse = dalloc<double>(ctx, ne + np);
            ctx->mse_n = ne + np;
        }
        if (ctx->mse_host.size() != ne + np) ctx->mse_host.assign(ne + np, 0.0);
        DSCE_HIP_CHECK(hipMemsetAsync(ctx->d_mse, 0, (ne + np) * sizeof(double), ctx->stream));
    }
}

static void set_mse_buffers(dsce_ctx* ctx) {
    if (!ctx->mse) return;
    const size_t ne = ctx->schemes.size() * ctx->nsnr * (ctx->niter + 1);
    ctx->buf.mse_err = ctx->d_mse;
    ctx->buf.mse_pow = ctx->d_mse + ne;
}

// the member's device MSE sums added into dst (the handle's host totals)
static void collect_mse(dsce_ctx* ctx, std::vector<double>& dst) {
    if (!ctx->mse) return;
    std::vector<double> h(ctx->mse_n);
    DSCE_HIP_CHECK(hipMemcpyAsync(h.data(), ctx->d_mse, h.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (dst.size() != h.size()) dst.assign(h.size(), 0.0);
    for (size_t i = 0; i < h.size(); ++i) dst[i] += h[i];
}

// Realisations [first_rep, first_rep + n_rep) of one member into its device
// counters (zeroed first); nothing is copied back
static void run_reps(dsce_ctx* ctx, uint64_t seed, uint64_t first_rep, uint64_t n_rep) {
    prepare_run(ctx);
    // any n_rep (the script's NrRepetitions, script:19 / :44): a tail that is no
    // multiple of 64 runs as a whole wave whose padding realisations count nothing
    uint64_t done = 0;
    while (done < n_rep) {
        const uint64_t left = n_rep - done;
        const int R = (int)std::min<uint64_t>((uint64_t)ctx->batch, (left + 63) / 64 * 64);
        const int nvalid = (int)std::min<uint64_t>((uint64_t)R, left);
        ensure_buffers(ctx, ctx->batch);
        set_mse_buffers(ctx);
        run_batch(ctx, seed, first_rep + done, R, nvalid, nullptr);
        done += (uint64_t)nvalid;
    }
}

// The member's device counters added into err_counts (null: none), its MSE sums
// into *mse_dst (the handle's totals), its timing events collected
static void finish_run(dsce_ctx* ctx, int64_t* err_counts, std::vector<double>* mse_dst) {
    const size_t n = err_counts ? ctx->counters_n : 0;
    if (n && ctx->h_counters_n < n) {
        if (ctx->h_counters) DSCE_HIP_CHECK(hipHostFree(ctx->h_counters));
        ctx->h_counters = nullptr;
        ctx->h_counters_n = 0;
        DSCE_HIP_CHECK(hipHostMalloc((void**)&ctx->h_counters, n * sizeof(unsigned long long), hipHostMallocDefault));
        ctx->h_counters_n = n;
    }
    if (n)
        DSCE_HIP_CHECK(hipMemcpyAsync(ctx->h_counters, ctx->d_counters, n * sizeof(unsigned long long),
                                      hipMemcpyDeviceToHost, ctx->stream));
    DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (ctx->timing) collect_timing(ctx);
    for (size_t i = 0; i < n; ++i) err_counts[i] += (int64_t)ctx->h_counters[i];
    if (mse_dst) collect_mse(ctx, *mse_dst);
}

// dsce_run of a multi-device context: one host thread per member on its slice,
// then one ncclAllReduce (sum) per buffer over the members' device counters /
// MSE sums (DSCE_REDUCE_RCCL) or the host sum (DSCE_REDUCE_HOST), and the total
// added into err_counts once
static void run_multi(dsce_ctx* ctx, uint64_t seed, uint64_t first_rep, uint64_t n_rep, int64_t* err_counts) {
    const size_t n = ctx->peers.size() + 1;
    std::vector<int> code(n, DSCE_OK);
    std::vector<std::string> msg(n);
    auto work = [&](size_t m) {
        dsce_ctx* c = member(ctx, m);
        try {
            check_ctx(c);
            uint64_t f = 0, k = 0;
            shard_slice(first_rep, n_rep, n, m, f, k);
            run_reps(c, seed, f, k);
            DSCE_HIP_CHECK(hipGetLastError());
            return;
        } catch (const ApiError& e) {
            code[m] = e.code;
            msg[m] = e.what();
        } catch (const HipError& e) {
            code[m] = DSCE_EHIP;
            msg[m] = e.what();
        } catch (const std::bad_alloc&) {
            code[m] = DSCE_ENOMEM;
            msg[m] = "host out of memory";
        } catch (const std::exception& e) {
            code[m] = DSCE_EINVAL;
            msg[m] = e.what();
        }
    };
    std::vector<std::thread> th;
    try {
        for (size_t m = 1; m < n; ++m) th.emplace_back(work, m);
    } catch (...) {
        for (auto& t : th) t.join();
        throw ApiError(DSCE_ENOMEM, "cannot start a member thread");
    }
    work(0);
    for (auto& t : th) t.join();
    for (size_t m = 0; m < n; ++m)
        if (code[m] != DSCE_OK) {
            // drain every member before reporting (no member's launches outlive the call)
            for (size_t j = 0; j < n; ++j) {
                (void)hipSetDevice(member(ctx, j)->device);
                (void)hipStreamSynchronize(member(ctx, j)->stream);
            }
            (void)hipSetDevice(ctx->device);
            throw ApiError(code[m], member_name(ctx, m) + ": " + msg[m]);
        }
    TraceRange trace_range(ctx->reduce == DSCE_REDUCE_RCCL ? "dsce counter all-reduce (rccl)" : "dsce counter sum (host)");
    if (ctx->reduce == DSCE_REDUCE_RCCL) {
        // stream-ordered behind each member's kernels; one group = one collective
        // launch per buffer and device
        // (the group is always closed, also when an enqueue fails: an open
        // group would swallow the next call's collectives)
        DSCE_NCCL_CHECK(ncclGroupStart());
        ncclResult_t first = ncclSuccess;
        for (size_t m = 0; m < n && first == ncclSuccess; ++m) {
            dsce_ctx* c = member(ctx, m);
            first = ncclAllReduce(c->d_counters, c->d_counters, c->counters_n, ncclUint64, ncclSum, ctx->comms[m],
                                  c->stream);
            if (first == ncclSuccess && c->mse)
                first = ncclAllReduce(c->d_mse, c->d_mse, c->mse_n, ncclFloat64, ncclSum, ctx->comms[m], c->stream);
        }
        const ncclResult_t end = ncclGroupEnd();
        DSCE_NCCL_CHECK(first);
        DSCE_NCCL_CHECK(end);
        for (size_t m = 1; m < n; ++m) {
            check_ctx(member(ctx, m));
            finish_run(member(ctx, m), nullptr, nullptr);
        }
        check_ctx(ctx);
        finish_run(ctx, err_counts, &ctx->mse_host);     // member 0 holds the sums
    } else {
        for (size_t m = 0; m < n; ++m) {
            check_ctx(member(ctx, m));
            finish_run(member(ctx, m), err_counts, &ctx->mse_host);
        }
        check_ctx(ctx);
    }
}

int dsce_run(dsce_ctx* ctx, uint64_t seed, uint64_t first_rep, uint64_t n_rep, int64_t* err_counts) {
    TraceRange trace_range("dsce_run");
    API_BEGIN
    check_ctx(ctx);
    if (!err_counts) throw ApiError(DSCE_EINVAL, "err_counts is null");
    if (!ctx->peers.empty() || ctx->reduce != DSCE_REDUCE_NONE) {
        run_multi(ctx, seed, first_rep, n_rep, err_counts);
    } else {
        run_reps(ctx, seed, first_rep, n_rep);
        finish_run(ctx, err_counts, &ctx->mse_host);
    }
    API_END
}

int dsce_bits_per_rep(dsce_ctx* ctx, int32_t id, int64_t* bits2) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!bits2) throw ApiError(DSCE_EINVAL, "null output");
    bits2[0] = s.bits_all;
    bits2[1] = s.bits_noedge;
    API_END
}

int dsce_channel_realise(dsce_ctx* ctx, uint64_t seed, uint64_t rep, double* ir_out) {
    API_BEGIN
    check_ctx(ctx);
    if (!ctx->chan_set) throw ApiError(DSCE_ESTATE, "dsce_set_channel first");
    if (!ir_out) throw ApiError(DSCE_EINVAL, "null output");
    // the realisation sits at lane rep % 8 of its batch, so the tests reach every
    // position of the kernels' realisation-to-wave mapping
    const int N = ctx->ch.N, R = 64, lane = (int)(rep % 8);
    double2* ir = dalloc<double2>(ctx, (size_t)ctx->ch.ntap * N * R);
    if (ctx->op.realise_win) {
        // only the samples the schemes' Q^H windows read (the run's Jakes kernels),
        // zero elsewhere
        if (ctx->jk_nsch != ctx->schemes.size()) update_jakes_chunks(ctx);
        update_jakes_groups(ctx);
        DSCE_HIP_CHECK(hipMemsetAsync(ir, 0, (size_t)ctx->ch.ntap * N * R * sizeof(double2), ctx->stream));
        launch_jakes(ctx->stream, ctx->op, ctx->ch, seed, rep - (uint64_t)lane, R, ir, &ctx->jk);
    } else {
        launch_jakes(ctx->stream, ctx->op, ctx->ch, seed, rep - (uint64_t)lane, R, ir);
    }
    std::vector<double2> h((size_t)ctx->ch.ntap * N * R);
    DSCE_HIP_CHECK(hipMemcpyAsync(h.data(), ir, h.size() * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
    DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    // by pointer: update_jakes_chunks / _groups above may have allocated after ir
    // (r04: popping the list's last entry freed ir twice at dsce_destroy and
    // dropped the Jakes groups from the list)
    free_alloc(ctx, ir);
    const int ntot = (int)ctx->pdp_norm.size();
    for (size_t i = 0; i < (size_t)N * ntot * 2; ++i) ir_out[i] = 0.0;
    for (int q = 0; q < ctx->ch.ntap; ++q)
        for (int n = 0; n < N; ++n) {
            const double2 v = h[((size_t)q * N + n) * R + lane];
            const size_t o = (size_t)ctx->ch.tap_delay[q] * N + n;
            ir_out[2 * o] = v.x;
            ir_out[2 * o + 1] = v.y;
        }
    API_END
}

int dsce_transmission_matrix(dsce_ctx* ctx, int32_t id, uint64_t seed, uint64_t rep, double* d_out) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!d_out) throw ApiError(DSCE_EINVAL, "null output");
    // the realisation at lane rep % 8 of a 64-realisation Jakes batch, every
    // sample formed (as dsce_channel_realise without realise_win)
    const int N = ctx->ch.N, R = 64, lane = (int)(rep % 8), LK = s.LK;
    std::vector<int> qlo(LK, 0), qhi(LK, 0);
    for (int c = 0; c < LK; ++c) {
        int lo = N, hi = 0;
        for (int n = 0; n < N; ++n)
            if (nz(s.Q[(size_t)c * N + n])) {
                lo = std::min(lo, n);
                hi = n + 1;
            }
        qlo[c] = lo < hi ? lo : 0;
        qhi[c] = hi;
    }
    std::vector<void*> tmp;
    auto talloc = [&](size_t bytes) {
        void* p;
        DSCE_HIP_CHECK(hipMalloc(&p, bytes ? bytes : 1));
        tmp.push_back(p);
        return p;
    };
    try {
        double2* ir = (double2*)talloc((size_t)ctx->ch.ntap * N * R * sizeof(double2));
        double2* G = (double2*)talloc((size_t)N * LK * sizeof(double2));
        double2* Q = (double2*)talloc((size_t)N * LK * sizeof(double2));
        double2* hg = (double2*)talloc((size_t)N * LK * sizeof(double2));
        double2* D = (double2*)talloc((size_t)LK * LK * sizeof(double2));
        int* dq = (int*)talloc(2 * (size_t)LK * sizeof(int));
        launch_jakes(ctx->stream, ctx->op, ctx->ch, seed, rep - (uint64_t)lane, R, ir);
        DSCE_HIP_CHECK(hipMemcpyAsync(G, s.G.data(), s.G.size() * sizeof(double2), hipMemcpyHostToDevice, ctx->stream));
        DSCE_HIP_CHECK(hipMemcpyAsync(Q, s.Q.data(), s.Q.size() * sizeof(double2), hipMemcpyHostToDevice, ctx->stream));
        DSCE_HIP_CHECK(hipMemcpyAsync(dq, qlo.data(), LK * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
        DSCE_HIP_CHECK(hipMemcpyAsync(dq + LK, qhi.data(), LK * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
        setup_transmission_matrix(ctx->stream, ctx->ch, LK, ir, R, lane, G, Q, dq, dq + LK, hg, D);
        DSCE_HIP_CHECK(hipGetLastError());
        DSCE_HIP_CHECK(hipMemcpyAsync(d_out, D, (size_t)LK * LK * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
        DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    } catch (...) {
        (void)hipStreamSynchronize(ctx->stream);
        for (void* p : tmp) (void)hipFree(p);
        throw;
    }
    for (void* p : tmp) DSCE_HIP_CHECK(hipFree(p));
    API_END
}

int dsce_get_correlation(dsce_ctx* ctx, int32_t id, double* r_hp, double* r_est, double* r_noi) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!s.mmse_ready) throw ApiError(DSCE_ESTATE, "dsce_build_mmse first");
    if (s.interp) throw ApiError(DSCE_ESTATE, "scheme uses an interpolation estimator (no correlation matrices)");
    if (r_hp) memcpy(r_hp, s.R_hP.data(), s.R_hP.size() * sizeof(double2));
    if (r_est) memcpy(r_est, s.R_est.data(), s.R_est.size() * sizeof(double2));
    if (r_noi) memcpy(r_noi, s.R_noI.data(), s.R_noI.size() * sizeof(double2));
    API_END
}

int dsce_tx_matrices(dsce_ctx* ctx, const dsce_tx_desc* d, double* G_out, double* Q_out) {
    API_BEGIN
    check_ctx(ctx);
    if (!d || d->n_subcarriers <= 0 || d->n_symbols <= 0 || d->n_samples <= 0 || d->fft_size <= 0 ||
        d->time_spacing <= 0 || (d->kind != 0 && d->kind != 1))
        throw ApiError(DSCE_EINVAL, "invalid tx description");
    if (d->kind == 1 && (!d->prototype || d->proto_len <= 0)) throw ApiError(DSCE_EINVAL, "FBMC needs the prototype");
    if (d->kind == 0 && d->time_spacing - d->cyclic_prefix != d->fft_size)
        throw ApiError(DSCE_EINVAL, "OFDM: time_spacing - cyclic_prefix must equal fft_size");
    TxDesc t{};
    t.kind = d->kind;
    t.L = d->n_subcarriers;
    t.K = d->n_symbols;
    t.N = d->n_samples;
    t.fft = d->fft_size;
    t.ifb = d->intermediate_bin;
    t.ts = d->time_spacing;
    t.cp = d->cyclic_prefix;
    t.zg = d->zero_guard;
    t.proto = d->proto_len;
    t.norm = d->norm;
    t.phase0 = d->initial_phase;
    t.rx_scale = d->rx_scale;
    const size_t n = (size_t)t.N * t.L * t.K;
    std::vector<void*> tmp;
    try {
        double* proto = nullptr;
        if (t.kind == 1) {
            DSCE_HIP_CHECK(hipMalloc((void**)&proto, t.proto * sizeof(double)));
            tmp.push_back(proto);
            DSCE_HIP_CHECK(hipMemcpy(proto, d->prototype, t.proto * sizeof(double), hipMemcpyHostToDevice));
        }
        double2 *G = nullptr, *Q = nullptr;
        if (G_out) {
            DSCE_HIP_CHECK(hipMalloc((void**)&G, n * sizeof(double2)));
            tmp.push_back(G);
        }
        if (Q_out) {
            DSCE_HIP_CHECK(hipMalloc((void**)&Q, n * sizeof(double2)));
            tmp.push_back(Q);
        }
        setup_tx_matrix(ctx->stream, t, proto, G, Q);
        DSCE_HIP_CHECK(hipGetLastError());
        if (G_out) DSCE_HIP_CHECK(hipMemcpyAsync(G_out, G, n * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
        if (Q_out) DSCE_HIP_CHECK(hipMemcpyAsync(Q_out, Q, n * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
        DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    } catch (...) {
        for (void* p : tmp) (void)hipFree(p);
        throw;
    }
    for (void* p : tmp) DSCE_HIP_CHECK(hipFree(p));
    API_END
}

int dsce_get_W(dsce_ctx* ctx, int32_t id, int32_t k, int32_t var, double* w_out) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!s.mmse_ready) throw ApiError(DSCE_ESTATE, "dsce_build_mmse first");
    if (!s.W) throw ApiError(DSCE_ESTATE, "scheme uses an interpolation estimator (no MMSE W)");
    if (k < 0 || k >= ctx->nsnr || var < 0 || var > 1 || !w_out) throw ApiError(DSCE_EINVAL, "bad W index");
    std::vector<double2> packed(s.w_elems);
    DSCE_HIP_CHECK(hipMemcpy(packed.data(), s.W + ((size_t)var * ctx->nsnr + k) * s.w_elems,
                             s.w_elems * sizeof(double2), hipMemcpyDeviceToHost));
    const size_t LK = s.LK, NP = s.d.n_pilots;
    memset(w_out, 0, LK * LK * NP * 2 * sizeof(double));
    const HostBand& b = s.wband;
    for (size_t blk = 0; blk < b.row0.size(); ++blk) {
        const int clo = b.klo[blk] / (int)NP, chi = b.khi[blk] / (int)NP;
        for (int rl = 0; rl < b.nrows[blk]; ++rl)
            for (int cc = clo; cc < chi; ++cc)
                for (size_t p = 0; p < NP; ++p) {
                    const double2 v = packed[b.off[blk] + ((size_t)(cc - clo) * NP + p) * b.rb + rl];
                    const size_t o = (size_t)(b.row0[blk] + rl) + LK * cc + LK * LK * p;
                    w_out[2 * o] = v.x;
                    w_out[2 * o + 1] = v.y;
                }
    }
    // the packed band holds D_hat's off-diagonal part; the diagonal is in Wd
    std::vector<double2> wd(LK * NP);
    DSCE_HIP_CHECK(hipMemcpy(wd.data(), s.Wd + ((size_t)var * ctx->nsnr + k) * LK * NP, wd.size() * sizeof(double2),
                             hipMemcpyDeviceToHost));
    for (size_t c = 0; c < LK; ++c)
        for (size_t p = 0; p < NP; ++p) {
            const size_t o = c + LK * c + LK * LK * p;
            w_out[2 * o] = wd[c * NP + p].x;
            w_out[2 * o + 1] = wd[c * NP + p].y;
        }
    API_END
}

int dsce_trace_unit_ex(dsce_ctx* ctx, int32_t id, uint64_t seed, uint64_t rep, int32_t k, const dsce_trace* out) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (k < 0 || k >= ctx->nsnr || !out) throw ApiError(DSCE_EINVAL, "bad trace arguments");
    prepare_run(ctx);
    ensure_buffers(ctx, ctx->batch);
    set_mse_buffers(ctx);
    const int LK = s.LK, ND = s.d.n_data, ns = ctx->niter + 1;
    std::vector<void*> tmp;
    auto talloc = [&](size_t bytes) {
        void* p;
        DSCE_HIP_CHECK(hipMalloc(&p, bytes));
        tmp.push_back(p);
        return p;
    };
    try {
        Trace tr{id, k, 0, out};
        tr.k.LK = LK;
        tr.k.ND = ND;
        tr.k.yest = (double2*)talloc((size_t)ns * LK * sizeof(double2));
        tr.k.yperf = (double2*)talloc((size_t)ns * LK * sizeof(double2));
        tr.k.hest = (double2*)talloc((size_t)ns * LK * sizeof(double2));
        tr.k.dec_e = (int*)talloc((size_t)ns * ND * sizeof(int));
        tr.k.dec_p = (int*)talloc((size_t)ns * ND * sizeof(int));
        tr.dev = (TraceK*)talloc(sizeof(TraceK));
        // all-ones bytes = NaN: "not written by any kernel" (0 is a legitimate value)
        DSCE_HIP_CHECK(hipMemsetAsync(tr.k.yest, 0xff, (size_t)ns * LK * sizeof(double2), ctx->stream));
        DSCE_HIP_CHECK(hipMemsetAsync(tr.k.yperf, 0xff, (size_t)ns * LK * sizeof(double2), ctx->stream));
        DSCE_HIP_CHECK(hipMemsetAsync(tr.k.hest, 0xff, (size_t)ns * LK * sizeof(double2), ctx->stream));
        // stages >= 1 of y_est / y_perf: NaN unless the host copies them from a
        // per-unit buffer (unfused paths) or a kernel writes them (fused paths)
        for (double* d : {out->yest_stages, out->yperf_stages})
            if (d)
                for (size_t i = 2 * (size_t)LK; i < 2 * (size_t)ns * LK; ++i) d[i] = std::nan("");
        DSCE_HIP_CHECK(hipMemsetAsync(tr.k.dec_e, 0xff, (size_t)ns * ND * sizeof(int), ctx->stream));
        DSCE_HIP_CHECK(hipMemsetAsync(tr.k.dec_p, 0xff, (size_t)ns * ND * sizeof(int), ctx->stream));
        // the unit sits at lane 0 of a 64-realisation batch starting at rep
        run_batch(ctx, seed, rep, 64, 64, &tr);
        std::vector<double2> ye((size_t)ns * LK), yp((size_t)ns * LK);
        DSCE_HIP_CHECK(hipMemcpyAsync(ye.data(), tr.k.yest, ye.size() * sizeof(double2), hipMemcpyDeviceToHost,
                                      ctx->stream));
        DSCE_HIP_CHECK(hipMemcpyAsync(yp.data(), tr.k.yperf, yp.size() * sizeof(double2), hipMemcpyDeviceToHost,
                                      ctx->stream));
        if (out->hest_stages)
            DSCE_HIP_CHECK(hipMemcpyAsync(out->hest_stages, tr.k.hest, (size_t)ns * LK * sizeof(double2),
                                          hipMemcpyDeviceToHost, ctx->stream));
        if (out->dec_est)
            DSCE_HIP_CHECK(hipMemcpyAsync(out->dec_est, tr.k.dec_e, (size_t)ns * ND * sizeof(int),
                                          hipMemcpyDeviceToHost, ctx->stream));
        if (out->dec_perf)
            DSCE_HIP_CHECK(hipMemcpyAsync(out->dec_perf, tr.k.dec_p, (size_t)ns * ND * sizeof(int),
                                          hipMemcpyDeviceToHost, ctx->stream));
        DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        // stage 0 of y_est / y_perf is y itself; a row of a later stage is what a
        // kernel wrote (NaN-initialised device trace), else what the host copied
        // from y_est / y_perf (unfused paths), else NaN (not formed: e.g. pilot
        // rows of the fused perfect-CSI chains)
        auto merge = [&](double* dst, const std::vector<double2>& dev) {
            if (!dst) return;
            for (int st = 1; st < ns; ++st)
                for (int r = 0; r < LK; ++r) {
                    const double2 v = dev[(size_t)st * LK + r];
                    double* d = dst + 2 * ((size_t)st * LK + r);
                    if (!std::isnan(v.x)) {
                        d[0] = v.x;
                        d[1] = v.y;
                    }
                }
        };
        merge(out->yest_stages, ye);
        merge(out->yperf_stages, yp);
        if (out->y) {
            for (double* d : {out->yest_stages, out->yperf_stages})
                if (d) memcpy(d, out->y, (size_t)LK * 2 * sizeof(double));
        }
        if (ctx->timing) collect_timing(ctx);
    } catch (...) {
        for (void* p : tmp) (void)hipFree(p);
        throw;
    }
    for (void* p : tmp) DSCE_HIP_CHECK(hipFree(p));
    API_END
}

int dsce_trace_unit(dsce_ctx* ctx, int32_t id, uint64_t seed, uint64_t rep, int32_t k, double* y, double* hp,
                    double* hest, double* h) {
    if (!y || !hp || !hest || !h) return api_fail(ctx, DSCE_EINVAL, "bad trace arguments");
    dsce_trace t{};
    t.y = y;
    t.hp_stages = hp;
    t.hest_stages = hest;
    t.h_perfect = h;
    return dsce_trace_unit_ex(ctx, id, seed, rep, k, &t);
}

int dsce_mmse_onetap(dsce_ctx* ctx, int32_t id, int32_t k, int32_t var, const double* hp_ls, int32_t n,
                     double* h_out) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!s.mmse_ready) throw ApiError(DSCE_ESTATE, "dsce_build_mmse first");
    if (k < 0 || k >= ctx->nsnr || var < 0 || var > 1 || n <= 0 || !hp_ls || !h_out)
        throw ApiError(DSCE_EINVAL, "bad dsce_mmse_onetap arguments");
    const int NP = s.d.n_pilots, LK = s.LK;
    double2* dh = nullptr;
    double2* dp = nullptr;
    DSCE_HIP_CHECK(hipMalloc(&dp, (size_t)NP * n * sizeof(double2)));
    try {
        DSCE_HIP_CHECK(hipMalloc(&dh, (size_t)LK * n * sizeof(double2)));
        DSCE_HIP_CHECK(hipMemcpyAsync(dp, hp_ls, (size_t)NP * n * sizeof(double2), hipMemcpyHostToDevice, ctx->stream));
        launch_mmse_onetap(ctx->stream, LK, NP, s.Wd + ((size_t)var * ctx->nsnr + k) * LK * NP, dp, n, dh);
        DSCE_HIP_CHECK(hipMemcpyAsync(h_out, dh, (size_t)LK * n * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
        DSCE_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    } catch (...) {
        (void)hipFree(dp);
        if (dh) (void)hipFree(dh);
        throw;
    }
    DSCE_HIP_CHECK(hipFree(dp));
    DSCE_HIP_CHECK(hipFree(dh));
    API_END
}

static int set_noise_slot_one(dsce_ctx* ctx, int32_t id, int32_t slot) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (slot < 0 || slot > 255) throw ApiError(DSCE_EINVAL, "noise slot must be 0..255");
    check_noise_streams(ctx, ctx->op.snr_base, ctx->nsnr, std::max(slot, max_noise_slot(ctx)));
    s.k.noise_slot = slot;
    API_END
}

int dsce_set_noise_slot(dsce_ctx* ctx, int32_t id, int32_t slot) {
    return fanout(ctx, [&](dsce_ctx* c) { return set_noise_slot_one(c, id, slot); });
}

static int set_interpolation_one(dsce_ctx* ctx, int32_t id, const double* I) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!I) throw ApiError(DSCE_EINVAL, "null interpolation matrix");
    const int LK = s.LK, NP = s.d.n_pilots;
    s.interp_I.assign((size_t)LK * NP, make_double2(0, 0));
    for (int c = 0; c < LK; ++c)
        for (int p = 0; p < NP; ++p) s.interp_I[(size_t)c * NP + p] = cx(I, (size_t)p * LK + c);   // column-major in
    if (s.W) {
        free_alloc(ctx, s.W);
        s.W = nullptr;
    }
    if (s.Wp3) free_alloc(ctx, s.Wp3);
    s.Wp3 = nullptr;
    s.interp = true;
    upload_interp(ctx, s);
    API_END
}

int dsce_set_interpolation(dsce_ctx* ctx, int32_t id, const double* I) {
    return fanout(ctx, [&](dsce_ctx* c) { return set_interpolation_one(c, id, I); });
}

static int enable_mse_one(dsce_ctx* ctx, int32_t enable) {
    API_BEGIN
    check_ctx(ctx);
    ctx->mse = enable != 0;
    ctx->mse_host.clear();
    API_END
}

int dsce_enable_mse(dsce_ctx* ctx, int32_t enable) {
    return fanout(ctx, [&](dsce_ctx* c) { return enable_mse_one(c, enable); });
}

int dsce_get_mse(dsce_ctx* ctx, double* err_sum, double* pow_sum) {
    API_BEGIN
    check_ctx(ctx);
    if (!ctx->mse) throw ApiError(DSCE_ESTATE, "dsce_enable_mse first");
    const size_t ns = ctx->schemes.size(), ne = ns * ctx->nsnr * (ctx->niter + 1), np = ns * ctx->nsnr;
    for (size_t i = 0; i < ne; ++i) {
        if (err_sum) err_sum[i] = ctx->mse_host.size() == ne + np ? ctx->mse_host[i] : 0.0;
    }
    for (size_t i = 0; i < np; ++i) {
        if (pow_sum) pow_sum[i] = ctx->mse_host.size() == ne + np ? ctx->mse_host[ne + i] : 0.0;
    }
    API_END
}

static int enable_timing_one(dsce_ctx* ctx, int32_t enable) {
    API_BEGIN
    check_ctx(ctx);
    ctx->timing = enable != 0;
    if (!ctx->timing) ctx->ktime.clear();
    API_END
}

int dsce_enable_timing(dsce_ctx* ctx, int32_t enable) {
    return fanout(ctx, [&](dsce_ctx* c) { return enable_timing_one(c, enable); });
}

int dsce_kernel_time(dsce_ctx* ctx, const char* kernel, int64_t* launches, double* total_ms) {
    API_BEGIN
    if (!ctx || !kernel) throw ApiError(DSCE_EINVAL, "null argument");
    auto it = ctx->ktime.find(kernel);
    if (launches) *launches = it == ctx->ktime.end() ? 0 : it->second.first;
    if (total_ms) *total_ms = it == ctx->ktime.end() ? 0.0 : it->second.second;
    API_END
}

int dsce_work_model(dsce_ctx* ctx, int32_t id, double* cmac, double* wbytes) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    // contraction CMACs over the band's off-diagonal pairs (the (r, r) pairs are
    // stored as zeros: D_hat - diag(D_hat) of script:482-484); with the fused MMSE
    // stage (OFDM) the same kernel also forms diag(D_hat) = Wd hP of the next
    // stage (LK x NP CMACs per unit)
    const double fused = (s.path & PATH_WPAIR3_FUSED) ? (double)s.LK * s.d.n_pilots : 0.0;
    if (cmac) *cmac = ((double)(s.w_struct - s.w_diag) + fused) * ctx->nsnr * ctx->niter;
    if (cmac && (s.path & PATH_MIC_STAGES)) {
        // k_mic_data (the bench's roofline kernel): dsce_kernel_work's model in CMACs
        *cmac = kernel_work(ctx, s, "k_mic_data").flops / 8.0;
    }
    if (wbytes) *wbytes = (double)s.w_elems * sizeof(double2);
    API_END
}

int dsce_kernel_work(dsce_ctx* ctx, const char* kernel, double* flops_per_rep, double* bytes_per_rep) {
    API_BEGIN
    check_ctx(ctx);
    if (!kernel) throw ApiError(DSCE_EINVAL, "null kernel name");
    const std::string n(kernel);
    double f = 0.0, b = 0.0;
    if (n == "k_jakes") {
        if (!ctx->schemes.empty()) {
            const KWork w = kernel_work(ctx, *ctx->schemes[0], n);
            f = w.flops;
            b = w.bytes;
        }
    } else {
        for (auto& sp : ctx->schemes) {
            const KWork w = kernel_work(ctx, *sp, n);
            f += w.flops;
            b += w.bytes;
        }
    }
    if (flops_per_rep) *flops_per_rep = f;
    if (bytes_per_rep) *bytes_per_rep = b;
    API_END
}

int dsce_structured_check(dsce_ctx* ctx, int32_t id, double* out) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!out) throw ApiError(DSCE_EINVAL, "null output");
    out[0] = s.mic_check;
    out[1] = s.mic_dev;
    out[2] = s.mic_wmax;
    out[3] = s.mic_rtol;
    out[4] = s.lr_resid;
    out[5] = s.Bz ? 1.0 : 0.0;
    out[6] = s.lr_ratio;
    API_END
}

int dsce_fp64_mfma_peak(dsce_ctx* ctx, double* tflops) {
    API_BEGIN
    check_ctx(ctx);
    if (!tflops) throw ApiError(DSCE_EINVAL, "null output");
    int cus = 0;
    DSCE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const int blocks = cus * 8, iters = 4096;          // 8 blocks x 4 waves per CU: 8 waves per SIMD
    double* out = dalloc<double>(ctx, (size_t)blocks * 256);
    hipEvent_t e0 = get_event(ctx), e1 = get_event(ctx);
    launch_mfma_f64_peak(ctx->stream, blocks, iters, out);     // warm-up (clocks up)
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        DSCE_HIP_CHECK(hipEventRecord(e0, ctx->stream));
        launch_mfma_f64_peak(ctx->stream, blocks, iters, out);
        DSCE_HIP_CHECK(hipEventRecord(e1, ctx->stream));
        DSCE_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        DSCE_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    DSCE_HIP_CHECK(hipGetLastError());
    ctx->event_pool.push_back(e0);
    ctx->event_pool.push_back(e1);
    free_alloc(ctx, out);
    *tflops = (double)blocks * 4 * iters * PEAK_MFMA_PER_ITER * 2048.0 / (best * 1e-3) / 1e12;
    API_END
}

// Kernel-selection options (Opts); the defaults are the measured-best path.
#define DSCE_OPTIONS(X)                                                                                  \
    X(xcd) X(fuse_stage) X(pic_chain) X(pfuse) X(stage_split) X(stage_rb) X(noise_fuse) \
    X(snr_chunk) X(jakes_rpw) X(wtrim) X(wcontract_valu) X(mmse_ic) X(jakes_win) X(txrx_fft) X(snr_base) X(jakes_mom) X(realise_win) X(tx_rows) X(pic_net) X(mic_net) X(mic_lr) X(pic_poly) X(wrow) X(jakes_grp2)

static int set_option_one(dsce_ctx* ctx, const char* name, int64_t value) {
    API_BEGIN
    check_ctx(ctx);
    if (!name) throw ApiError(DSCE_EINVAL, "null option name");
    const std::string n(name);
    int* slot = nullptr;
#define X(f) if (n == #f) slot = &ctx->op.f;
    DSCE_OPTIONS(X)
#undef X
    if (!slot && (n == "pic_skip" || n == "ic_streams"))
        throw ApiError(DSCE_EINVAL, "option '" + n + "' was retired in r06 (measured neutral in r04 / r05; DESIGN.md 2.0d, 2.0f)");
    if (!slot) throw ApiError(DSCE_EINVAL, "unknown option '" + n + "'");
    if (n == "stage_rb" && value != 4 && value != 8 && value != 16) throw ApiError(DSCE_EINVAL, "stage_rb: 4 | 8 | 16");
    if (n == "jakes_rpw" && value != 1 && value != 2) throw ApiError(DSCE_EINVAL, "jakes_rpw: 1 | 2");
    if (n == "pic_chain" && value != 0 && value != 3)
        throw ApiError(DSCE_EINVAL, "pic_chain: 0 (per-iteration passes) | 3 (k_pic_fft); the r01 chains 1 / 2 "
                                    "(k_pic_chain, k_pic_mfma) were retired in r03");
    if (n == "snr_base" && (value < 0 || value > 255)) throw ApiError(DSCE_EINVAL, "snr_base: 0..255");
    if (n == "snr_base") check_noise_streams(ctx, value, ctx->nsnr, max_noise_slot(ctx));
    if (value < -1 || value > 1 << 20) throw ApiError(DSCE_EINVAL, "option value out of range");
    *slot = (int)value;
    API_END
}

int dsce_set_option(dsce_ctx* ctx, const char* name, int64_t value) {
    return fanout(ctx, [&](dsce_ctx* c) { return set_option_one(c, name, value); });
}

int dsce_get_option(dsce_ctx* ctx, const char* name, int64_t* value) {
    API_BEGIN
    if (!ctx || !name || !value) throw ApiError(DSCE_EINVAL, "null argument");
    const std::string n(name);
    const int* slot = nullptr;
#define X(f) if (n == #f) slot = &ctx->op.f;
    DSCE_OPTIONS(X)
#undef X
    if (!slot) throw ApiError(DSCE_EINVAL, "unknown option '" + n + "'");
    *value = *slot;
    API_END
}
#undef DSCE_OPTIONS

int dsce_path_info(dsce_ctx* ctx, int32_t id, uint32_t* flags) {
    API_BEGIN
    check_ctx(ctx);
    Scheme& s = get_scheme(ctx, id);
    if (!flags) throw ApiError(DSCE_EINVAL, "null output");
    *flags = s.path;
    API_END
}

int dsce_scheme_dims(dsce_ctx* ctx, int32_t id, dsce_dims* dims) {
    API_BEGIN
    if (!ctx) throw ApiError(DSCE_EINVAL, "null context");
    Scheme& s = get_scheme(ctx, id);
    if (!dims) throw ApiError(DSCE_EINVAL, "null output");
    dims->n_samples = s.N;
    dims->n_taps = (int32_t)ctx->pdp_norm.size();
    dims->lk = s.LK;
    dims->n_pilots = s.d.n_pilots;
    dims->n_data = s.d.n_data;
    dims->n_tx_symbols = s.d.n_tx_symbols;
    dims->n_schemes = (int32_t)ctx->schemes.size();
    dims->n_snr = ctx->nsnr;
    dims->n_iter = ctx->niter;
    dims->n_counters = (int64_t)ctx->schemes.size() * 4 * ctx->nsnr * (ctx->niter + 1);
    API_END
}

}  // extern "C"
