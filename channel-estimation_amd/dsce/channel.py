"""Host-side mirror of the reference's ``+Channel/FastFading.m``.

Only the constructor's parameter processing runs on the host
(PDP tables and sample-grid quantisation, FastFading.m:47-131, 186-190).
The per-realisation work — ``NewRealization`` (Jakes sum of sinusoids,
FastFading.m:222-238) and ``GetConvolutionMatrix`` (FastFading.m:276-295) —
is executed by the HIP engine (``k_jakes`` in csrc/kernels_mc.hip) when the
object is bound to an :class:`dsce.engine.Engine`; the realisation index plays
the role of MATLAB's implicit RNG state (counter-based Philox, see
``include/dsce.h``).
"""
from __future__ import annotations

import numpy as np

# FastFading.m:56-107 — (relative power dB, delay s)
_PDP_TABLES = {
    "Flat": ([0.0], [0.0]),
    "AWGN": ([0.0], [0.0]),
    "PedestrianA": ([0, -9.7, -19.2, -22.8], [0, 110e-9, 190e-9, 410e-9]),
    "PedestrianB": ([0, -0.9, -4.9, -8, -7.8, -23.9], [0, 200e-9, 800e-9, 1200e-9, 2300e-9, 3700e-9]),
    "VehicularA": ([0, -1, -9, -10, -15, -20], [0, 310e-9, 710e-9, 1090e-9, 1730e-9, 2510e-9]),
    "VehicularB": ([-2.5, 0, -12.8, -10, -25.2, -16], [0, 300e-9, 8900e-9, 12900e-9, 17100e-9, 20000e-9]),
    "ExtendedPedestrianA": ([0, -1, -2, -3, -8, -17.2, -20.8], [0, 30e-9, 70e-9, 90e-9, 110e-9, 190e-9, 410e-9]),
    "ExtendedVehicularA": ([0, -1.5, -1.4, -3.6, -0.6, -9.1, -7, -12, -16.9],
                           [0, 30e-9, 150e-9, 310e-9, 370e-9, 710e-9, 1090e-9, 1730e-9, 2510e-9]),
}
_TDL = {
    "TDL-A": ([-13.4, 0, -2.2, -4, -6, -8.2, -9.9, -10.5, -7.5, -15.9, -6.6, -16.7, -12.4, -15.2, -10.8, -11.3,
               -12.7, -16.2, -18.3, -18.9, -16.6, -19.9, -29.7],
              [0.0000, 0.3819, 0.4025, 0.5868, 0.4610, 0.5375, 0.6708, 0.5750, 0.7618, 1.5375, 1.8978, 2.2242,
               2.1718, 2.4942, 2.5119, 3.0582, 4.0810, 4.4579, 4.5695, 4.7966, 5.0066, 5.3043, 9.6586]),
    "TDL-B": ([0, -2.2, -4, -3.2, -9.8, -1.2, -3.4, -5.2, -7.6, -3, -8.9, -9, -4.8, -5.7, -7.5, -1.9, -7.6, -12.2,
               -9.8, -11.4, -14.9, -9.2, -11.3],
              [0.0000, 0.1072, 0.2155, 0.2095, 0.2870, 0.2986, 0.3752, 0.5055, 0.3681, 0.3697, 0.5700, 0.5283,
               1.1021, 1.2756, 1.5474, 1.7842, 2.0169, 2.8294, 3.0219, 3.6187, 4.1067, 4.2790, 4.7834]),
    "TDL-C": ([-4.4, -1.2, -3.5, -5.2, -2.5, 0, -2.2, -3.9, -7.4, -7.1, -10.7, -11.1, -5.1, -6.8, -8.7, -13.2,
               -13.9, -13.9, -15.8, -17.1, -16, -15.7, -21.6, -22.8],
              [0, 0.2099, 0.2219, 0.2329, 0.2176, 0.6366, 0.6448, 0.6560, 0.6584, 0.7935, 0.8213, 0.9336, 1.2285,
               1.3083, 2.1704, 2.7105, 4.2589, 4.6003, 5.4902, 5.6077, 6.3065, 6.6374, 7.0427, 8.6523]),
}


def quantise_pdp(pdp, sampling_rate):
    """Power-delay profile on the sample grid, FastFading.m:47-131.

    Returns ``(PowerDelayProfile, PowerDelayProfileNormalized)``, both indexed by
    tap delay in samples (tap 0 = no delay).
    """
    dt = 1.0 / sampling_rate
    if isinstance(pdp, str):
        name = pdp
        if name[:3] == "TDL":
            pos1 = name.index("_")
            pos2 = name.index("ns")
            rms = float(name[pos1 + 1:pos2]) * 1e-9
            name = name[:5]
            pw, dl = _TDL[name]
            dl = [rms * d for d in dl]
        elif name in _PDP_TABLES:
            pw, dl = _PDP_TABLES[name]
        else:
            raise ValueError("Power delay profile model not supported!")
        pw = np.asarray(pw, dtype=float)
        dl = np.asarray(dl, dtype=float)
        idx = (np.sign(dl / dt) * np.floor(np.abs(dl / dt) + 0.5)).astype(np.int64)   # MATLAB round               # 0-based (FastFading.m:111 is 1-based)
        tmp = np.zeros((idx.size, int(idx.max()) + 1))
        for i in range(idx.size):
            tmp[i, idx[i]] = 10.0 ** (pw[i] / 10)
        profile = tmp.sum(axis=0)
    else:
        profile = np.asarray(pdp, dtype=float).reshape(-1)
    return profile, profile / profile.sum()


class FastFading:
    """``Channel.FastFading(SR, PDP, N, fD, DopplerModel, Paths, nTx, nRx, warn)``
    (FastFading.m:25-192), single antenna (1x1).  Engine-backed Doppler models:
    'Jakes' / 'Uniform' (sum of sinusoids, FastFading.m:222-238),
    'Discrete-Jakes' / 'Discrete-Uniform' (IFFT of the discrete Doppler
    spectrum, FastFading.m:158-177, :203-221) and MaximumDopplerShift == 0
    (time-invariant block fading, FastFading.m:241-246; with the 'Flat' PDP the
    doubly-flat channel of SimpleVersion_DoublyFlat.m:123)."""

    MODELS = {"Jakes": 0, "Uniform": 1, "Discrete-Jakes": 2, "Discrete-Uniform": 3}

    def __init__(self, SamplingRate, PowerDelayProfile, SamplesTotal, MaximumDopplerShift,
                 DopplerModel, Paths, nTxAntennas=1, nRxAntennas=1, WarningIfSampleRateDoesNotMatch=False):
        if nTxAntennas != 1 or nRxAntennas != 1:
            raise ValueError("only the 1x1 channel used by DoublySelectiveChannelEstimation.m is provided")
        self.SamplingRate = float(SamplingRate)
        self.SamplesTotal = int(SamplesTotal)
        self.MaximumDopplerShift = float(MaximumDopplerShift)
        self.DopplerModel = DopplerModel
        self.Paths = int(Paths)
        self.dt = 1.0 / self.SamplingRate
        if PowerDelayProfile == "AWGN":
            self.MaximumDopplerShift = 0.0
        self.PowerDelayProfile, self.PowerDelayProfileNormalized = quantise_pdp(PowerDelayProfile, self.SamplingRate)
        self.IndexDelayTaps = np.flatnonzero(self.PowerDelayProfile)   # FastFading.m:131 (0-based)
        if DopplerModel not in self.MODELS:
            raise ValueError("Doppler spectrum not supported: %s" % DopplerModel)
        self.UseDiscreteDopplerSpectrum = False
        if DopplerModel.startswith("Discrete") and self.MaximumDopplerShift > 0:
            df = self.SamplingRate / self.SamplesTotal
            if self.MaximumDopplerShift / df <= 0.5:               # FastFading.m:153-156
                self.MaximumDopplerShift = 0.0
            else:                                                  # FastFading.m:158-177
                self.UseDiscreteDopplerSpectrum = True
                nd = int(np.ceil(self.MaximumDopplerShift / df))
                ip = df * (np.arange(-nd - 1, nd + 1) + 0.5)
                ip = np.clip(ip, -self.MaximumDopplerShift, self.MaximumDopplerShift)
                if DopplerModel == "Discrete-Jakes":
                    S = np.arcsin(ip[1:] / self.MaximumDopplerShift) - np.arcsin(ip[:-1] / self.MaximumDopplerShift)
                else:
                    S = ip[1:] - ip[:-1]
                self.DiscreteDopplerSpectrum = S / S.sum()
        self._engine = None
        self._rep = 0
        self._seed = 0

    @property
    def Ltap(self):
        return self.PowerDelayProfile.size

    def GetTimeCorrelation(self):
        """FastFading.m:321-340 (Jakes: J0, Uniform: sinc).  For a discrete
        Doppler spectrum the reference assigns no TimeCorrelation (its switch
        only knows 'Jakes' / 'Uniform', :331-336), so this raises like MATLAB."""
        from scipy.special import j0
        N = self.SamplesTotal
        t = self.dt * np.arange(-(N - 1), N)
        if self.MaximumDopplerShift <= 0:
            return np.ones(2 * N - 1), t
        if self.DopplerModel.startswith("Discrete"):
            raise ValueError("TimeCorrelation is not defined for a discrete Doppler spectrum (FastFading.m:321-336)")
        if self.DopplerModel == "Jakes":
            return j0(np.pi * 2 * self.MaximumDopplerShift * t), t
        return np.sinc(2 * self.MaximumDopplerShift * t), t

    # -- engine-backed hot path --------------------------------------------
    def bind(self, engine, seed=0):
        self._engine = engine
        self._seed = int(seed)
        self._rep = 0

    def NewRealization(self):
        """Advance to the next realisation (counter-based RNG: rep index += 1)."""
        self._rep += 1

    @property
    def ImpulseResponse(self):
        if self._engine is None:
            raise RuntimeError("FastFading is not bound to an engine (call bind())")
        return self._engine.channel_impulse_response(self._seed, self._rep)

    def GetConvolutionMatrix(self):
        """Sparse N x N convolution matrix H[n, n-tau] = IR[n, tau] (FastFading.m:276-295)."""
        import scipy.sparse as sp
        ir = self.ImpulseResponse            # (N, Ltap) complex
        N = self.SamplesTotal
        rows, cols, vals = [], [], []
        for tau in self.IndexDelayTaps:
            n = np.arange(tau, N)
            rows.append(n)
            cols.append(n - tau)
            vals.append(ir[n, tau])
        H = sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(N, N))
        return [[H]]
