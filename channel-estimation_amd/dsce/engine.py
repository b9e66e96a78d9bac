"""ctypes binding of the C-ABI in include/dsce.h (libdsce.so, HIP for gfx950).

This is the Python twin of the MEX gateway described in INTEGRATION.md: it
converts the host objects (dsce.configs.Scheme, dsce.channel.FastFading) into
the plain column-major interleaved-complex buffers of the ABI.  There is no
CPU fallback: if the shared library is missing or no GPU is present the calls
raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSCE_LIB", os.path.join(_HERE, "libdsce.so"))

EXPORTED = [
    "dsce_abi_version", "dsce_device_count", "dsce_create", "dsce_destroy", "dsce_last_error",
    "dsce_set_channel", "dsce_set_snr", "dsce_add_scheme", "dsce_build_mmse", "dsce_set_batch", "dsce_run",
    "dsce_bits_per_rep", "dsce_channel_realise", "dsce_get_correlation", "dsce_get_W", "dsce_trace_unit",
    "dsce_enable_timing", "dsce_kernel_time", "dsce_work_model", "dsce_mmse_onetap", "dsce_tx_matrices",
    "dsce_set_noise_slot", "dsce_set_interpolation", "dsce_enable_mse", "dsce_get_mse", "dsce_trace_unit_ex",
    "dsce_scheme_dims", "dsce_path_info", "dsce_set_option", "dsce_get_option", "dsce_fp64_mfma_peak",
    "dsce_kernel_work", "dsce_structured_check", "dsce_create_multi", "dsce_group_info",
    "dsce_transmission_matrix",
]

ABI_VERSION = 7

# dsce_group_info reduce kinds (include/dsce.h DSCE_REDUCE_*)
REDUCE = {0: "none", 1: "rccl", 2: "host"}

# dsce_path_info bits (include/dsce.h DSCE_PATH_*)
PATH_BITS = {
    "wpair3_fused": 1 << 0, "wpair3": 1 << 1, "wpair4m": 1 << 2, "wcontract_valu": 1 << 3, "pic_mfma": 1 << 4,
    "pic_chain": 1 << 5, "pic_passes": 1 << 6, "stage_fused": 1 << 7, "stage_split": 1 << 8, "noise_fused": 1 << 9,
    "pic_fft": 1 << 10, "mic_fft": 1 << 11, "txrx_fft": 1 << 12, "pilot_fused": 1 << 13, "mic_stages": 1 << 14,
    "mic_lr": 1 << 15, "pic_poly": 1 << 16, "wrow3": 1 << 17,
}


class ChannelDesc(C.Structure):
    _fields_ = [("n_samples", C.c_int32), ("n_taps", C.c_int32), ("sampling_rate", C.c_double),
                ("max_doppler", C.c_double), ("n_paths", C.c_int32), ("doppler_model", C.c_int32),
                ("pdp_norm", C.POINTER(C.c_double))]


class SchemeDesc(C.Structure):
    _fields_ = [("n_subcarriers", C.c_int32), ("n_symbols", C.c_int32), ("n_tx_symbols", C.c_int32),
                ("n_pilots", C.c_int32), ("n_data", C.c_int32), ("mod_order", C.c_int32),
                ("bits_per_symbol", C.c_int32), ("despread", C.c_int32), ("real_detect", C.c_int32),
                ("bits_slot", C.c_int32), ("pilot_slot", C.c_int32), ("kappa", C.c_double),
                ("data_div", C.c_double), ("G", C.POINTER(C.c_double)), ("Q", C.POINTER(C.c_double)),
                ("P", C.POINTER(C.c_double)), ("pilot_pos", C.POINTER(C.c_int32)),
                ("data_pos", C.POINTER(C.c_int32)), ("considered", C.POINTER(C.c_uint8)),
                ("symbols", C.POINTER(C.c_double))]


class Dims(C.Structure):
    _fields_ = [("n_samples", C.c_int32), ("n_taps", C.c_int32), ("lk", C.c_int32), ("n_pilots", C.c_int32),
                ("n_data", C.c_int32), ("n_tx_symbols", C.c_int32), ("n_schemes", C.c_int32), ("n_snr", C.c_int32),
                ("n_iter", C.c_int32), ("n_counters", C.c_int64)]


class Trace(C.Structure):
    _fields_ = [("y", C.POINTER(C.c_double)), ("h_perfect", C.POINTER(C.c_double)),
                ("hp_stages", C.POINTER(C.c_double)), ("hest_stages", C.POINTER(C.c_double)),
                ("yest_stages", C.POINTER(C.c_double)), ("yperf_stages", C.POINTER(C.c_double)),
                ("dec_est", C.POINTER(C.c_int32)), ("dec_perf", C.POINTER(C.c_int32))]


class TxDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("n_subcarriers", C.c_int32), ("n_symbols", C.c_int32),
                ("n_samples", C.c_int32), ("fft_size", C.c_int32), ("intermediate_bin", C.c_int32),
                ("time_spacing", C.c_int32), ("cyclic_prefix", C.c_int32), ("zero_guard", C.c_int32),
                ("proto_len", C.c_int32), ("norm", C.c_double), ("initial_phase", C.c_double),
                ("rx_scale", C.c_double), ("prototype", C.POINTER(C.c_double))]


_lib = None


def load_library(path=None):
    """Load libdsce.so (raises OSError with a build hint when it is missing)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise OSError("libdsce.so not found at %s — build it with `make -C channel-estimation_amd` "
                      "(or __graft_entry__.build())" % p)
    lib = C.CDLL(p)
    vp = C.c_void_p
    dp = C.POINTER(C.c_double)
    i64p = C.POINTER(C.c_int64)
    lib.dsce_abi_version.restype = C.c_int
    lib.dsce_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.dsce_create.argtypes = [C.c_int, C.POINTER(vp)]
    lib.dsce_create_multi.argtypes = [C.POINTER(C.c_int32), C.c_int32, C.POINTER(vp)]
    lib.dsce_group_info.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.dsce_destroy.argtypes = [vp]
    lib.dsce_destroy.restype = C.c_int
    lib.dsce_last_error.argtypes = [vp]
    lib.dsce_last_error.restype = C.c_char_p
    lib.dsce_set_channel.argtypes = [vp, C.POINTER(ChannelDesc)]
    lib.dsce_set_snr.argtypes = [vp, dp, C.c_int32, C.c_int32]
    lib.dsce_add_scheme.argtypes = [vp, C.POINTER(SchemeDesc), C.POINTER(C.c_int32)]
    lib.dsce_build_mmse.argtypes = [vp, C.c_double]
    lib.dsce_set_batch.argtypes = [vp, C.c_int32]
    lib.dsce_run.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint64, i64p]
    lib.dsce_bits_per_rep.argtypes = [vp, C.c_int32, i64p]
    lib.dsce_channel_realise.argtypes = [vp, C.c_uint64, C.c_uint64, dp]
    lib.dsce_get_correlation.argtypes = [vp, C.c_int32, dp, dp, dp]
    lib.dsce_transmission_matrix.argtypes = [vp, C.c_int32, C.c_uint64, C.c_uint64, dp]
    lib.dsce_get_W.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, dp]
    lib.dsce_trace_unit.argtypes = [vp, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32, dp, dp, dp, dp]
    lib.dsce_enable_timing.argtypes = [vp, C.c_int32]
    lib.dsce_kernel_time.argtypes = [vp, C.c_char_p, i64p, dp]
    lib.dsce_work_model.argtypes = [vp, C.c_int32, dp, dp]
    lib.dsce_mmse_onetap.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, dp, C.c_int32, dp]
    lib.dsce_tx_matrices.argtypes = [vp, C.POINTER(TxDesc), dp, dp]
    lib.dsce_set_noise_slot.argtypes = [vp, C.c_int32, C.c_int32]
    lib.dsce_set_interpolation.argtypes = [vp, C.c_int32, dp]
    lib.dsce_enable_mse.argtypes = [vp, C.c_int32]
    lib.dsce_get_mse.argtypes = [vp, dp, dp]
    lib.dsce_trace_unit_ex.argtypes = [vp, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32, C.POINTER(Trace)]
    lib.dsce_scheme_dims.argtypes = [vp, C.c_int32, C.POINTER(Dims)]
    lib.dsce_path_info.argtypes = [vp, C.c_int32, C.POINTER(C.c_uint32)]
    lib.dsce_set_option.argtypes = [vp, C.c_char_p, C.c_int64]
    lib.dsce_get_option.argtypes = [vp, C.c_char_p, C.POINTER(C.c_int64)]
    lib.dsce_fp64_mfma_peak.argtypes = [vp, dp]
    lib.dsce_kernel_work.argtypes = [vp, C.c_char_p, dp, dp]
    lib.dsce_structured_check.argtypes = [vp, C.c_int32, dp]
    for name in EXPORTED:
        fn = getattr(lib, name)
        if name != "dsce_last_error":
            fn.restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def _cplx(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.complex128).reshape(-1, order="F"))
    return a


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class DsceError(RuntimeError):
    pass


class Engine:
    """One engine context = one GPU + one HIP stream (dsce_create), or, with a
    sequence of devices, one multi-device context (dsce_create_multi, ABI 7):
    every configuration call reaches every member, run() shards the
    realisations over the members and sums their counters with one in-library
    RCCL all-reduce (host sum when a device repeats)."""

    def __init__(self, device=0, lib_path=None):
        self.lib = load_library(lib_path)
        h = C.c_void_p()
        if isinstance(device, (list, tuple, np.ndarray)):
            devs = np.ascontiguousarray(device, dtype=np.int32)
            rc = self.lib.dsce_create_multi(devs.ctypes.data_as(C.POINTER(C.c_int32)), int(devs.size), C.byref(h))
            what = "dsce_create_multi(devices=%s)" % list(devs)
        else:
            rc = self.lib.dsce_create(int(device), C.byref(h))
            what = "dsce_create(device=%d)" % device
        if rc != 0 or not h.value:
            raise DsceError("%s failed with %d (no HIP device?)" % (what, rc))
        self.h = h
        self._keep = []
        self.schemes = []
        self.nsnr = 0
        self.niter = 0
        self.N = None
        self.ntaps = None

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.dsce_last_error(self.h)
            raise DsceError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def close(self):
        """dsce_destroy; raises DsceError when a HIP call of the teardown failed
        (ABI 6; the context is freed either way)."""
        if getattr(self, "h", None) is not None and self.h.value:
            rc = self.lib.dsce_destroy(self.h)
            self.h = None
            if rc != 0:
                raise DsceError("dsce_destroy failed (%d): a HIP call of the teardown failed (see stderr)" % rc)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- configuration -------------------------------------------------------
    def set_channel(self, ff):
        pdp = np.ascontiguousarray(ff.PowerDelayProfileNormalized, dtype=np.float64)
        self._keep.append(pdp)
        d = ChannelDesc(ff.SamplesTotal, pdp.size, ff.SamplingRate, ff.MaximumDopplerShift, ff.Paths,
                        ff.MODELS[ff.DopplerModel], _dptr(pdp))
        self._chk(self.lib.dsce_set_channel(self.h, C.byref(d)), "dsce_set_channel")
        self.N = ff.SamplesTotal
        self.ntaps = pdp.size

    def set_snr(self, pn_time, n_iter):
        pn = np.ascontiguousarray(pn_time, dtype=np.float64)
        self._chk(self.lib.dsce_set_snr(self.h, _dptr(pn), pn.size, int(n_iter)), "dsce_set_snr")
        self.nsnr = pn.size
        self.niter = int(n_iter)

    def add_scheme(self, sc):
        G = _cplx(sc.G)
        Q = _cplx(sc.Q)
        P = _cplx(sc.P)
        pil = np.ascontiguousarray(sc.pilot_pos, dtype=np.int32)
        dat = np.ascontiguousarray(sc.data_pos, dtype=np.int32)
        cons = np.ascontiguousarray(sc.considered_symbols, dtype=np.uint8)
        sym = _cplx(sc.const.SymbolMapping)
        self._keep += [G, Q, P, pil, dat, cons, sym]
        L = sc.extras.get("pilot_matrix").shape[0] if "pilot_matrix" in sc.extras else sc.LK
        d = SchemeDesc(L, sc.LK // L, sc.P.shape[1], sc.n_pilots, sc.n_data, sc.const.ModulationOrder,
                       sc.bits_per_symbol, int(sc.despread), int(sc.real_detect), sc.bits_slot, sc.pilot_slot,
                       sc.kappa, sc.data_div, _dptr(G), _dptr(Q), _dptr(P),
                       pil.ctypes.data_as(C.POINTER(C.c_int32)), dat.ctypes.data_as(C.POINTER(C.c_int32)),
                       cons.ctypes.data_as(C.POINTER(C.c_uint8)), _dptr(sym))
        sid = C.c_int32()
        self._chk(self.lib.dsce_add_scheme(self.h, C.byref(d), C.byref(sid)), "dsce_add_scheme")
        self.schemes.append(sc)
        return sid.value

    def set_noise_slot(self, sid, slot):
        """Schemes of one slot share the AWGN draw (dsce_set_noise_slot)."""
        self._chk(self.lib.dsce_set_noise_slot(self.h, int(sid), int(slot)), "dsce_set_noise_slot")

    def set_interpolation(self, sid, interp):
        """One-tap estimate h_hat = interp @ hP (LK x NP) instead of the MMSE W
        (dsce_set_interpolation; PSACE ChannelInterpolation weights)."""
        sc = self.schemes[sid]
        I = _cplx(np.asarray(interp).reshape(sc.LK, sc.n_pilots))
        self._keep.append(I)
        self._chk(self.lib.dsce_set_interpolation(self.h, int(sid), _dptr(I)), "dsce_set_interpolation")

    def build_mmse(self, zero_threshold=1e-8):
        self._chk(self.lib.dsce_build_mmse(self.h, float(zero_threshold)), "dsce_build_mmse")

    def set_batch(self, reps):
        self._chk(self.lib.dsce_set_batch(self.h, int(reps)), "dsce_set_batch")

    # -- Monte Carlo -----------------------------------------------------------
    def counter_shape(self):
        return (len(self.schemes), 2, 2, self.nsnr, 1 + self.niter)

    def run(self, seed, first_rep, n_rep, counts=None):
        if counts is None:
            counts = np.zeros(self.counter_shape(), dtype=np.int64)
        assert counts.dtype == np.int64 and counts.flags.c_contiguous and counts.shape == self.counter_shape()
        self._chk(self.lib.dsce_run(self.h, int(seed), int(first_rep), int(n_rep),
                                    counts.ctypes.data_as(C.POINTER(C.c_int64))), "dsce_run")
        return counts

    def bits_per_rep(self, sid):
        b = np.zeros(2, dtype=np.int64)
        self._chk(self.lib.dsce_bits_per_rep(self.h, int(sid), b.ctypes.data_as(C.POINTER(C.c_int64))),
                  "dsce_bits_per_rep")
        return b

    # -- setup producers (row f1) ----------------------------------------------
    def tx_matrices(self, mod):
        """(G, Q) of a dsce.modulation.OFDM / FBMC object computed on the GPU:
        G = mod.GetTXMatrix(), Q = mod.GetRXMatrix()' (script:191-195)."""
        from dsce.modulation import FBMC, OFDM
        Nr, Impl, PHY = mod.Nr, mod.Implementation, mod.PHY
        L, K, N = Nr.Subcarriers, Nr.MCSymbols, Nr.SamplesTotal
        proto = None
        if isinstance(mod, OFDM):
            if PHY.TransmitRealSignal:
                raise DsceError("GetTXMatrix is not supported for PHY.TransmitRealSignal == true")
            d = TxDesc(0, L, K, N, Impl.FFTSize, Impl.IntermediateFrequency, Impl.TimeSpacing, Impl.CyclicPrefix,
                       Impl.ZeroGuardSamples, 0, Impl.NormalizationFactor, 0.0,
                       L * PHY.SubcarrierSpacing / PHY.SamplingRate, None)
        elif isinstance(mod, FBMC):
            if PHY.TransmitRealSignal:
                raise DsceError("real-signal FBMC is not supported")
            proto = np.ascontiguousarray(mod.PrototypeFilter.TimeDomain, dtype=np.float64)
            d = TxDesc(1, L, K, N, Impl.FFTSize, Impl.IntermediateFrequency, Impl.TimeSpacing, 0, 0, proto.size,
                       Impl.NormalizationFactor, Impl.InitialPhaseShift, L / (PHY.SamplingRate * PHY.TimeSpacing),
                       _dptr(proto))
        else:
            raise TypeError("OFDM or FBMC object expected")
        G = np.zeros(2 * N * L * K)
        Q = np.zeros(2 * N * L * K)
        self._chk(self.lib.dsce_tx_matrices(self.h, C.byref(d), _dptr(G), _dptr(Q)), "dsce_tx_matrices")
        shape = (N, L * K)
        return (G.view(np.complex128).reshape(shape, order="F"), Q.view(np.complex128).reshape(shape, order="F"))

    # -- probes ----------------------------------------------------------------
    def channel_impulse_response(self, seed, rep):
        out = np.zeros(2 * self.N * self.ntaps)
        self._chk(self.lib.dsce_channel_realise(self.h, int(seed), int(rep), _dptr(out)), "dsce_channel_realise")
        return out.view(np.complex128).reshape(self.N, self.ntaps, order="F")

    def transmission_matrix(self, sid, seed, rep):
        """D = Q^H H G (LK x LK) of realisation `rep` (dsce_transmission_matrix,
        script:381-393)."""
        LK = self.schemes[sid].LK
        out = np.zeros(2 * LK * LK)
        self._chk(self.lib.dsce_transmission_matrix(self.h, int(sid), int(seed), int(rep), _dptr(out)),
                  "dsce_transmission_matrix")
        return out.view(np.complex128).reshape(LK, LK, order="F")

    def correlation(self, sid):
        NP = self.schemes[sid].n_pilots
        rhp = np.zeros(2 * NP * NP)
        rest = np.zeros(2 * self.nsnr * NP * NP)
        rnoi = np.zeros(2 * self.nsnr * NP * NP)
        self._chk(self.lib.dsce_get_correlation(self.h, int(sid), _dptr(rhp), _dptr(rest), _dptr(rnoi)),
                  "dsce_get_correlation")
        f = lambda a, n: a.view(np.complex128).reshape(n, NP, NP).transpose(0, 2, 1)   # column-major NP x NP
        return f(rhp, 1)[0], f(rest, self.nsnr), f(rnoi, self.nsnr)

    def W(self, sid, snr_index, variant=0):
        sc = self.schemes[sid]
        out = np.zeros(2 * sc.LK * sc.LK * sc.n_pilots)
        self._chk(self.lib.dsce_get_W(self.h, int(sid), int(snr_index), int(variant), _dptr(out)), "dsce_get_W")
        return out.view(np.complex128)

    def trace_unit(self, sid, seed, rep, snr_index):
        """Every stage of one (rep, SNR) unit through the same kernels as run()
        (dsce_trace_unit_ex): y, h (= diag D), and per stage hp (LS pilots), hest
        (diag D_hat), yest / yperf (IC inputs; row 0 = y) and the detected symbol
        indices dec_e / dec_p (-1 where the path forms no decision)."""
        d = self.scheme_dims(sid)
        ns, LK, NP, ND = d.n_iter + 1, d.lk, d.n_pilots, d.n_data
        bufs = dict(y=np.zeros(2 * LK), h=np.zeros(2 * LK), hp=np.zeros(2 * ns * NP), hest=np.zeros(2 * ns * LK),
                    yest=np.zeros(2 * ns * LK), yperf=np.zeros(2 * ns * LK))
        dec_e = np.zeros(ns * ND, dtype=np.int32)
        dec_p = np.zeros(ns * ND, dtype=np.int32)
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))
        t = Trace(_dptr(bufs["y"]), _dptr(bufs["h"]), _dptr(bufs["hp"]), _dptr(bufs["hest"]), _dptr(bufs["yest"]),
                  _dptr(bufs["yperf"]), ip(dec_e), ip(dec_p))
        self._chk(self.lib.dsce_trace_unit_ex(self.h, int(sid), int(seed), int(rep), int(snr_index), C.byref(t)),
                  "dsce_trace_unit_ex")
        v = lambda a: a.view(np.complex128)
        return dict(y=v(bufs["y"]), h=v(bufs["h"]), hp=v(bufs["hp"]).reshape(ns, NP),
                    hest=v(bufs["hest"]).reshape(ns, LK), yest=v(bufs["yest"]).reshape(ns, LK),
                    yperf=v(bufs["yperf"]).reshape(ns, LK), dec_e=dec_e.reshape(ns, ND), dec_p=dec_p.reshape(ns, ND))

    # -- engine state ------------------------------------------------------------
    def scheme_dims(self, sid):
        d = Dims()
        self._chk(self.lib.dsce_scheme_dims(self.h, int(sid), C.byref(d)), "dsce_scheme_dims")
        return d

    def path_info(self, sid):
        """Names of the kernel paths the scheme's last run / trace went through."""
        f = C.c_uint32()
        self._chk(self.lib.dsce_path_info(self.h, int(sid), C.byref(f)), "dsce_path_info")
        return {k for k, bit in PATH_BITS.items() if f.value & bit}

    def set_option(self, name, value):
        self._chk(self.lib.dsce_set_option(self.h, name.encode(), int(value)), "dsce_set_option(%s)" % name)

    def get_option(self, name):
        v = C.c_int64()
        self._chk(self.lib.dsce_get_option(self.h, name.encode(), C.byref(v)), "dsce_get_option(%s)" % name)
        return v.value

    def mmse_onetap(self, sid, snr_index, hp_ls, variant=0):
        """h_hat = diag(sum_p W_p hP_p) for LS vectors hp_ls (NP,) or (NP, n)."""
        sc = self.schemes[sid]
        hp = np.asarray(hp_ls, dtype=np.complex128)
        one = hp.ndim == 1
        hp = np.ascontiguousarray(hp.reshape(sc.n_pilots, -1).T)      # n x NP rows = column-major NP x n
        n = hp.shape[0]
        out = np.zeros(2 * sc.LK * n)
        self._chk(self.lib.dsce_mmse_onetap(self.h, int(sid), int(snr_index), int(variant),
                                            hp.ctypes.data_as(C.POINTER(C.c_double)), n, _dptr(out)),
                  "dsce_mmse_onetap")
        h = out.view(np.complex128).reshape(n, sc.LK).T
        return h[:, 0] if one else h

    # -- channel-estimation MSE (build-defined) ---------------------------------
    def enable_mse(self, on=True):
        """Start (and reset) the MSE sums of dsce_run (dsce_enable_mse)."""
        self._chk(self.lib.dsce_enable_mse(self.h, int(bool(on))), "dsce_enable_mse")

    def mse(self):
        """(err [scheme][snr][stage] = sum |h_hat - h|^2, pow [scheme][snr] = sum |h|^2)
        since enable_mse(); NMSE = err / pow[..., None]."""
        ns = len(self.schemes)
        err = np.zeros((ns, self.nsnr, 1 + self.niter))
        pw = np.zeros((ns, self.nsnr))
        self._chk(self.lib.dsce_get_mse(self.h, _dptr(err), _dptr(pw)), "dsce_get_mse")
        return err, pw

    def group_info(self):
        """(devices, reduce) of the context (dsce_group_info): the members' HIP
        devices and how run() sums them ('none' | 'rccl' | 'host')."""
        n = C.c_int32()
        self._chk(self.lib.dsce_group_info(self.h, C.byref(n), None, None), "dsce_group_info")
        devs = np.zeros(n.value, dtype=np.int32)
        red = C.c_int32()
        self._chk(self.lib.dsce_group_info(self.h, None, devs.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(red)),
                  "dsce_group_info")
        return [int(d) for d in devs], REDUCE.get(red.value, str(red.value))

    # -- measurement -----------------------------------------------------------
    def enable_timing(self, on=True):
        self._chk(self.lib.dsce_enable_timing(self.h, int(bool(on))), "dsce_enable_timing")

    def kernel_time(self, name):
        n = C.c_int64()
        ms = C.c_double()
        self._chk(self.lib.dsce_kernel_time(self.h, name.encode(), C.byref(n), C.byref(ms)), "dsce_kernel_time")
        return n.value, ms.value

    def fp64_mfma_peak(self):
        """Measured FP64 matrix-core peak of this GPU, TFLOP/s (dsce_fp64_mfma_peak)."""
        t = C.c_double()
        self._chk(self.lib.dsce_fp64_mfma_peak(self.h, C.byref(t)), "dsce_fp64_mfma_peak")
        return t.value

    def kernel_work(self, name):
        """(flops, bytes) per realisation of timed kernel group `name` (dsce_kernel_work;
        0 = not modelled for the path that ran)."""
        f = C.c_double()
        b = C.c_double()
        self._chk(self.lib.dsce_kernel_work(self.h, name.encode(), C.byref(f), C.byref(b)), "dsce_kernel_work")
        return f.value, b.value

    def structured_check(self, sid):
        """build_mic's guard of the structured MMSE IC (dsce_structured_check): dict with
        ratio (kept iff <= 1: the worst slice's deviation over its rounding bar
        min(1e-9, max(1e-11, 4e-16 kappa(R))) max|W|), dev (max |Q' H_hat G - W_thr|),
        wmax (max |W|), rtol (the largest per-slice bar), and the low-rank tap
        operator's fit residual lr_resid (relative), lr (built and kept: eligible; a
        run uses it with options mic_lr = 1 and mic_net bit 0, see path_info's
        mic_lr) and lr_ratio (capped bar min(1e-9, max(1e-13, 4e-16 kappa(R))))."""
        out = (C.c_double * 7)()
        self._chk(self.lib.dsce_structured_check(self.h, int(sid), out), "dsce_structured_check")
        return dict(ratio=out[0], dev=out[1], wmax=out[2], rtol=out[3], lr_resid=out[4], lr=bool(out[5]),
                    lr_ratio=out[6])

    def work_model(self, sid):
        cm = C.c_double()
        wb = C.c_double()
        self._chk(self.lib.dsce_work_model(self.h, int(sid), C.byref(cm), C.byref(wb)), "dsce_work_model")
        return cm.value, wb.value


def gpu_tx(device=0):
    """Producer of (G, Q) for build_setup(tx=...): dsce_tx_matrices on `device`
    (row f1, OFDM.m:184-218 / FBMC.m:318-354 in closed form per element)."""
    def produce(mod):
        eng = Engine(device)
        try:
            return eng.tx_matrices(mod)
        finally:
            eng.close()
    return produce


def build_engine(setup, schemes=None, device=0, zero_threshold=None, batch=None, options=None):
    """Engine configured like the script: channel, SNR list, schemes, MMSE setup.
    ``options``: dsce_set_option name -> value, applied before the MMSE build."""
    eng = Engine(device)
    for k, v in (options or {}).items():
        eng.set_option(k, v)
    eng.set_channel(setup.channel)
    eng.set_snr(setup.pn_time, setup.n_iter)
    names = list(setup.schemes) if schemes is None else list(schemes)
    for n in names:
        eng.add_scheme(setup.schemes[n])
    eng.build_mmse(setup.zero_threshold if zero_threshold is None else zero_threshold)
    if batch:
        eng.set_batch(batch)
    return eng
