"""Host-side mirror of the reference's ``+Modulation`` package (setup producers).

These classes keep the constructor signatures and method names of the MATLAB
classes so a user of the reference finds the same surface:

* ``FBMC``  — ``+Modulation/FBMC.m:28-59`` (ctor), ``:61-160``
  (SetDependentParameters), ``:255-315`` (polyphase Modulation/Demodulation),
  ``:318-354`` (GetTXMatrix/GetRXMatrix), ``:355-400`` (GetFBMCMatrix,
  GetInterferenceMatrix), ``:629-706`` (Hermite prototype).
* ``OFDM``  — ``+Modulation/OFDM.m:23-88`` (ctor + dependent parameters),
  ``:153-181`` (Modulation/Demodulation), ``:184-218`` (GetTXMatrix/GetRXMatrix).
* ``SignalConstellation`` — ``+Modulation/SignalConstellation.m:24-101``.

They run once per run on the host (fp64 numpy): they produce the operators
(G, Q, constellation tables) that are handed to the HIP engine through the
C-ABI (``include/dsce.h``).  Nothing here is on the per-realisation hot path.
All vectors that the reference indexes column-major (``x(:)``) are flattened
with ``order='F'`` here as well.
"""
from __future__ import annotations

import numpy as np


def _col(x):
    return np.asarray(x).reshape(-1, order="F")


def mround(x):
    """MATLAB round (half away from zero); Python's round is half-to-even."""
    return float(np.sign(x) * np.floor(abs(x) + 0.5))


# --------------------------------------------------------------------------
# FBMC
# --------------------------------------------------------------------------
def _hermite_h(n, x):
    """Hermite polynomials, FBMC.m:685-706."""
    if n == 0:
        return np.ones_like(x)
    if n == 4:
        return 12 + (-48) * x**2 + 16 * x**4
    if n == 8:
        return 1680 + (-13440) * x**2 + 13440 * x**4 + (-3584) * x**6 + 256 * x**8
    if n == 12:
        return (665280 + (-7983360) * x**2 + 13305600 * x**4 + (-7096320) * x**6
                + 1520640 * x**8 + (-135168) * x**10 + 4096 * x**12)
    if n == 16:
        return (518918400 + (-8302694400) * x**2 + 19372953600 * x**4
                + (-15498362880) * x**6 + 5535129600 * x**8 + (-984023040) * x**10
                + 89456640 * x**12 + (-3932160) * x**14 + 65536 * x**16)
    if n == 20:
        return (670442572800 + (-13408851456000) * x**2 + 40226554368000 * x**4
                + (-42908324659200) * x**6 + 21454162329600 * x**8
                + (-5721109954560) * x**10 + 866834841600 * x**12
                + (-76205260800) * x**14 + 3810263040 * x**16 + (-99614720) * x**18
                + 1048576 * x**20)
    raise ValueError(n)


def prototype_filter_hermite(T0, dt, OF):
    """FBMC.m:629-647.  Time grid ``-(OF*T0):dt:(OF*T0-dt)``."""
    n = int(mround(2 * OF * T0 / dt))
    t = -(OF * T0) + np.arange(n) * dt
    z = np.sqrt(2 * np.pi) * (t / (T0 / np.sqrt(2)))
    g = np.exp(-np.pi * (t / (T0 / np.sqrt(2))) ** 2) / np.sqrt(T0)
    coef = {0: 1.412692577, 4: -3.0145e-3, 8: -8.8041e-6, 12: -2.2611e-9,
            16: -4.4570e-15, 20: 1.8633e-16}
    p = np.zeros(n)
    for order in (0, 4, 8, 12, 16, 20):
        p = p + g * _hermite_h(order, z) * coef[order]
    return p / np.sqrt(np.sum(np.abs(p) ** 2) * dt)


class _NS:
    """Attribute bag standing in for the MATLAB struct properties (Nr, PHY, ...)."""

    def __repr__(self):
        return "%s(%s)" % (type(self).__name__, ", ".join(
            "%s=%r" % kv for kv in sorted(vars(self).items()) if np.isscalar(kv[1])))


class FBMC:
    """``Modulation.FBMC(L, K, F, SR, IF, RealSig, Method, O, Phase, Polyphase)``
    (FBMC.m:28-59).  Only the 'Hermite-OQAM' prototype used by every BASELINE
    configuration is supported; other methods raise like the reference's
    ``otherwise`` branch would for an unknown method (FBMC.m:129-130)."""

    def __init__(self, *args):
        if len(args) == 10:
            (L, K, F, SR, IF, real_sig, method, O, phase, poly) = args
        elif len(args) == 0:
            L, K, F = 12, 30, 15e3
            SR, IF, real_sig, method, O, phase, poly = L * F, 0, False, "Hermite-OQAM", 8, 0, True
        else:
            raise ValueError("Number of input variables must be either 0 (default values) or 10")
        self.Nr = _NS()
        self.PHY = _NS()
        self.PrototypeFilter = _NS()
        self.Implementation = _NS()
        self.Nr.Subcarriers = int(L)
        self.Nr.MCSymbols = int(K)
        self.PHY.SubcarrierSpacing = float(F)
        self.PHY.SamplingRate = float(SR)
        self.PHY.IntermediateFrequency = float(IF)
        self.PHY.TransmitRealSignal = bool(real_sig)
        self.Method = method
        self.PrototypeFilter.OverlappingFactor = int(O)
        self.Implementation.InitialPhaseShift = float(phase)
        self.Implementation.UsePolyphase = bool(poly)
        self.SetDependentParameters()

    def SetDependentParameters(self):
        """FBMC.m:61-160 (Hermite-OQAM branch)."""
        PHY, Nr, Impl, PF = self.PHY, self.Nr, self.Implementation, self.PrototypeFilter
        if (PHY.SamplingRate / (2 * PHY.SubcarrierSpacing)) % 1 != 0:
            PHY.SubcarrierSpacing = PHY.SamplingRate / (2 * mround(PHY.SamplingRate / (2 * PHY.SubcarrierSpacing)))
        if (PHY.IntermediateFrequency / PHY.SubcarrierSpacing) % 1 != 0:
            PHY.IntermediateFrequency = mround(PHY.IntermediateFrequency / PHY.SubcarrierSpacing) * PHY.SubcarrierSpacing
        if PHY.SamplingRate < Nr.Subcarriers * PHY.SubcarrierSpacing:
            raise ValueError("Sampling Rate must be higher: at least Number of Subcarriers times Subcarrier Spacing")
        PHY.dt = 1.0 / PHY.SamplingRate
        if self.Method != "Hermite-OQAM":
            raise ValueError('Method (prototype filter) "%s" is not supported' % self.Method)
        Impl.TimeSpacing = int(mround(PHY.SamplingRate / (2 * PHY.SubcarrierSpacing)))
        PHY.TimeSpacing = Impl.TimeSpacing * PHY.dt
        Impl.FrequencySpacing = PF.OverlappingFactor
        PF.TimeDomain = prototype_filter_hermite(PHY.TimeSpacing * 2, PHY.dt, PF.OverlappingFactor / 2)
        Nr.SamplesPrototypeFilter = PF.TimeDomain.size
        Nr.SamplesTotal = Nr.SamplesPrototypeFilter + (Nr.MCSymbols - 1) * Impl.TimeSpacing
        l, k = np.meshgrid(np.arange(Nr.Subcarriers), np.arange(Nr.MCSymbols), indexing="ij")
        Impl.PhaseShift = np.exp(1j * np.pi / 2 * (l + k)) * np.exp(1j * Impl.InitialPhaseShift)
        Impl.FFTSize = int(mround(Nr.SamplesPrototypeFilter / Impl.FrequencySpacing))
        Impl.IntermediateFrequency = int(mround(PHY.IntermediateFrequency / PHY.SubcarrierSpacing))
        rows = (np.arange(Nr.Subcarriers) + Impl.IntermediateFrequency) % Impl.FFTSize
        pm = np.zeros((Impl.FFTSize, Nr.MCSymbols), dtype=bool)
        pm[rows, :] = True
        Impl.IndexPolyphaseMap = pm
        Impl.NormalizationFactor = np.sqrt(PHY.SamplingRate**2 / PHY.SubcarrierSpacing**2
                                           * PHY.TimeSpacing / Nr.Subcarriers)

    # -- modulation (polyphase, FBMC.m:255-285 / 287-315) ------------------
    def Modulation(self, DataSymbols):
        Nr, Impl, PF = self.Nr, self.Implementation, self.PrototypeFilter
        X = np.asarray(DataSymbols, dtype=complex).reshape(Nr.Subcarriers, Nr.MCSymbols, order="F")
        tmp = np.zeros((Impl.FFTSize, Nr.MCSymbols), dtype=complex)
        # logical-index assignment, column-major (FBMC.m:264)
        tmp.T[Impl.IndexPolyphaseMap.T] = _col(X * Impl.PhaseShift * Impl.NormalizationFactor)
        if self.PHY.TransmitRealSignal:
            tmp = (tmp + np.conj(tmp[np.r_[0, Impl.FFTSize - 1:0:-1], :])) / np.sqrt(2)
        blk = np.tile(np.fft.ifft(tmp, axis=0), (Impl.FrequencySpacing, 1)) * PF.TimeDomain[:, None]
        s = np.zeros(Nr.SamplesTotal, dtype=complex)
        for k in range(Nr.MCSymbols):
            s[k * Impl.TimeSpacing:k * Impl.TimeSpacing + Nr.SamplesPrototypeFilter] += blk[:, k]
        return s

    def Demodulation(self, ReceivedSignal):
        Nr, Impl, PF = self.Nr, self.Implementation, self.PrototypeFilter
        r = _col(ReceivedSignal)
        idx = np.arange(Nr.SamplesPrototypeFilter)[:, None] + Impl.TimeSpacing * np.arange(Nr.MCSymbols)[None, :]
        filt = r[idx] * PF.TimeDomain[:, None]
        folded = filt.reshape(Impl.FFTSize, Impl.FrequencySpacing, Nr.MCSymbols, order="F").sum(axis=1)
        tmp = np.fft.fft(folded, axis=0)
        if self.PHY.TransmitRealSignal:
            tmp = tmp * np.sqrt(2)
        sel = tmp.T[Impl.IndexPolyphaseMap.T].reshape(Nr.MCSymbols, Nr.Subcarriers).T
        return sel * np.conj(Impl.PhaseShift) / (Impl.NormalizationFactor * self.PHY.SubcarrierSpacing)

    # -- matrix description (FBMC.m:318-400) --------------------------------
    def GetTXMatrix(self):
        Nr, Impl = self.Nr, self.Implementation
        L, K = Nr.Subcarriers, Nr.MCSymbols
        temp = np.zeros((Nr.SamplesTotal, L), dtype=complex)
        x = np.zeros((L, K), dtype=complex)
        for l in range(L):
            x[l, 0] = 1
            temp[:, l] = self.Modulation(x)
            x[l, 0] = 0
        G = np.zeros((Nr.SamplesTotal, L * K), dtype=complex)
        for k in range(K):
            G[:, k * L:(k + 1) * L] = np.roll(temp, k * Impl.TimeSpacing, axis=0) * (1j ** k)
        return G

    def GetRXMatrix(self):
        return self.GetTXMatrix().conj().T * (self.Nr.Subcarriers / (self.PHY.SamplingRate * self.PHY.TimeSpacing))

    def GetInterferenceMatrix(self):
        L, K = self.Nr.Subcarriers, self.Nr.MCSymbols
        d = np.zeros((L, K))
        d[0, 0] = 1
        Y11 = self.Demodulation(self.Modulation(d)).reshape(L, K, order="F")
        l_all, k_all = np.meshgrid(np.arange(L), np.arange(K), indexing="ij")
        Y11 = Y11 * (np.exp(1j * np.pi / 2 * (l_all + k_all)) * np.exp(-1j * np.pi * k_all * (l_all / 2)))
        top = np.hstack([Y11[:0:-1, :0:-1], Y11[:0:-1, :]])
        bot = np.hstack([Y11[:, :0:-1], Y11])
        return np.vstack([top, bot])

    def GetFBMCMatrix(self):
        """FastCalculation branch, FBMC.m:359-377 (OQAM phase correction)."""
        L, K = self.Nr.Subcarriers, self.Nr.MCSymbols
        IM = self.GetInterferenceMatrix()
        sub, sym = np.meshgrid(np.arange(1, L + 1), np.arange(1, K + 1), indexing="ij")
        sub, sym = _col(sub), _col(sym)
        dsub = sub[:, None] - sub[None, :]
        dsym = sym[:, None] - sym[None, :]
        isub = np.repeat((sub - 1)[:, None], L * K, axis=1)
        rows = dsub + L - 1
        cols = dsym + K - 1
        D = IM[rows, cols]
        tf = self.PHY.TimeSpacing * self.PHY.SubcarrierSpacing
        return D * np.exp(-1j * np.pi / 2 * (dsub + dsym)) * np.exp(-1j * 2 * np.pi * tf * dsym * (isub + dsub / 2))


# --------------------------------------------------------------------------
# OFDM
# --------------------------------------------------------------------------
class OFDM:
    """``Modulation.OFDM(L, K, F, SR, IF, RealSig, CP_s, ZG_s)`` (OFDM.m:23-51)."""

    def __init__(self, *args):
        if len(args) == 8:
            L, K, F, SR, IF, real_sig, cp, zg = args
        elif len(args) == 0:
            L, K, F, SR, IF, real_sig, cp, zg = 24, 14, 15e3, 15e3 * 24 * 14, 0, False, 1 / (14 * 15e3), 0
        else:
            raise ValueError("Number of input variables must be either 0 (default values) or 8")
        self.Nr = _NS()
        self.PHY = _NS()
        self.Implementation = _NS()
        self.Nr.Subcarriers = int(L)
        self.Nr.MCSymbols = int(K)
        self.PHY.SubcarrierSpacing = float(F)
        self.PHY.SamplingRate = float(SR)
        self.PHY.IntermediateFrequency = float(IF)
        self.PHY.TransmitRealSignal = bool(real_sig)
        self.PHY.CyclicPrefixLength = float(cp)
        self.PHY.ZeroGuardTimeLength = float(zg)
        self.SetDependentParameters()

    def SetDependentParameters(self):
        """OFDM.m:53-88."""
        PHY, Nr, Impl = self.PHY, self.Nr, self.Implementation
        if (mround(PHY.SamplingRate / PHY.SubcarrierSpacing * 1e5) / 1e5) % 1 != 0:
            PHY.SubcarrierSpacing = PHY.SamplingRate / mround(PHY.SamplingRate / PHY.SubcarrierSpacing)
        if (mround(PHY.IntermediateFrequency / PHY.SubcarrierSpacing * 1e5) / 1e5) % 1 != 0:
            PHY.IntermediateFrequency = mround(PHY.IntermediateFrequency / PHY.SubcarrierSpacing) * PHY.SubcarrierSpacing
        if PHY.SamplingRate < Nr.Subcarriers * PHY.SubcarrierSpacing:
            raise ValueError("Sampling theorem is not fullfilled")
        if abs((mround(PHY.CyclicPrefixLength * PHY.SamplingRate * 1e5) / 1e5) % 1) != 0:
            PHY.CyclicPrefixLength = mround(PHY.CyclicPrefixLength * PHY.SamplingRate) / PHY.SamplingRate
        Impl.CyclicPrefix = int(mround(PHY.CyclicPrefixLength * PHY.SamplingRate))
        Impl.ZeroGuardSamples = int(mround(PHY.ZeroGuardTimeLength * PHY.SamplingRate))
        Impl.TimeSpacing = int(mround(PHY.SamplingRate / PHY.SubcarrierSpacing)) + Impl.CyclicPrefix
        Impl.FFTSize = int(mround(PHY.SamplingRate / PHY.SubcarrierSpacing))
        Impl.IntermediateFrequency = int(mround(PHY.IntermediateFrequency / PHY.SubcarrierSpacing))
        Impl.NormalizationFactor = np.sqrt(PHY.SamplingRate**2 / PHY.SubcarrierSpacing**2 / Nr.Subcarriers)
        PHY.dt = 1.0 / PHY.SamplingRate
        PHY.TimeSpacing = Impl.TimeSpacing * PHY.dt
        Nr.SamplesTotal = Nr.MCSymbols * Impl.TimeSpacing + 2 * Impl.ZeroGuardSamples

    def Modulation(self, DataSymbols):
        Nr, Impl = self.Nr, self.Implementation
        X = np.asarray(DataSymbols, dtype=complex).reshape(Nr.Subcarriers, Nr.MCSymbols, order="F")
        tmp = np.zeros((Impl.FFTSize, Nr.MCSymbols), dtype=complex)
        tmp[Impl.IntermediateFrequency + np.arange(Nr.Subcarriers), :] = X * Impl.NormalizationFactor
        if self.PHY.TransmitRealSignal:
            tmp = (tmp + np.conj(tmp[np.r_[0, Impl.FFTSize - 1:0:-1], :])) / np.sqrt(2)
        t = np.fft.ifft(tmp, axis=0)
        cp = Impl.CyclicPrefix
        body = np.vstack([t[t.shape[0] - cp:, :], t]) if cp > 0 else t
        zg = np.zeros(Impl.ZeroGuardSamples, dtype=complex)
        return np.concatenate([zg, _col(body), zg])

    def Demodulation(self, ReceivedSignal):
        Nr, Impl = self.Nr, self.Implementation
        r = _col(ReceivedSignal)
        zg = Impl.ZeroGuardSamples
        body = r[zg:r.size - zg].reshape(Impl.TimeSpacing, Nr.MCSymbols, order="F")
        tmp = np.fft.fft(body[Impl.CyclicPrefix:, :], axis=0)
        if self.PHY.TransmitRealSignal:
            tmp = tmp * np.sqrt(2)
        return tmp[Impl.IntermediateFrequency + np.arange(Nr.Subcarriers), :] / Impl.NormalizationFactor

    def GetTXMatrix(self):
        if self.PHY.TransmitRealSignal:
            raise ValueError("GetTXMatrix is not supported for PHY.TransmitRealSignal == true!")
        Nr, Impl = self.Nr, self.Implementation
        L, K = Nr.Subcarriers, Nr.MCSymbols
        temp = np.zeros((Nr.SamplesTotal, L), dtype=complex)
        x = np.zeros((L, K), dtype=complex)
        for l in range(L):
            x[l, 0] = 1
            temp[:, l] = self.Modulation(x)
            x[l, 0] = 0
        G = np.zeros((Nr.SamplesTotal, L * K), dtype=complex)
        for k in range(K):
            G[:, k * L:(k + 1) * L] = np.roll(temp, k * Impl.TimeSpacing, axis=0)
        return G

    def CPSampleMask(self):
        """Boolean mask of the samples that GetRXMatrix zeroes (OFDM.m:216-217)."""
        Impl = self.Implementation
        m = np.zeros(self.Nr.SamplesTotal, dtype=bool)
        idx = Impl.ZeroGuardSamples + np.arange(Impl.CyclicPrefix)[:, None] + \
            np.arange(self.Nr.MCSymbols)[None, :] * Impl.TimeSpacing
        m[_col(idx)] = True
        return m

    def GetRXMatrix(self):
        Q = self.GetTXMatrix().conj().T * (self.Nr.Subcarriers * self.PHY.SubcarrierSpacing / self.PHY.SamplingRate)
        Q[:, self.CPSampleMask()] = 0
        return Q


# --------------------------------------------------------------------------
# Signal constellation
# --------------------------------------------------------------------------
def _bi2de(bits):
    """Communications-toolbox ``bi2de`` default: first column is the LSB."""
    bits = np.asarray(bits, dtype=np.int64)
    return (bits * (1 << np.arange(bits.shape[1]))[None, :]).sum(axis=1)


class SignalConstellation:
    """``Modulation.SignalConstellation(M, 'QAM'|'PAM')`` (SignalConstellation.m:24-74)."""

    def __init__(self, ModulationOrder, Method):
        M = int(ModulationOrder)
        self.ModulationOrder = M
        self.Method = Method
        if Method == "QAM":
            sq = int(mround(np.sqrt(M)))
            atom = np.zeros((sq, int(np.log2(sq))), dtype=bool)
            atom[:sq // 2, 0] = True
            for i in range(1, atom.shape[1]):
                t = atom[0::2, i - 1]
                atom[:, i] = np.concatenate([t, t[::-1]])
            IQ = 2 * np.arange(1, sq + 1) - sq - 1
            I_rep, Q_rep = np.meshgrid(IQ, IQ)          # MATLAB meshgrid semantics
            I_rep, Q_rep = _col(I_rep), _col(Q_rep)
            sym = I_rep + 1j * Q_rep
            sym = sym / np.sqrt(np.mean(np.abs(sym) ** 2))
            bm = np.zeros((M, int(np.log2(M))), dtype=bool)
            for x in IQ:
                bm[np.ix_(I_rep == x, np.arange(1, bm.shape[1], 2))] = atom
                bm[np.ix_(Q_rep == x, np.arange(0, bm.shape[1], 2))] = atom
        elif Method == "PAM":
            bm = np.zeros((M, int(np.log2(M))), dtype=bool)
            bm[:M // 2, 0] = True
            for i in range(1, bm.shape[1]):
                t = bm[0::2, i - 1]
                bm[:, i] = np.concatenate([t, t[::-1]])
            sym = (2 * np.arange(1, M + 1) - M - 1).astype(float)
            sym = sym / np.sqrt(np.mean(np.abs(sym) ** 2))
            sym = sym.astype(complex)
        else:
            raise ValueError("Signal constellation method must be QAM or PAM!")
        order = np.argsort(_bi2de(bm), kind="stable")
        self.SymbolMapping = sym[order]
        self.BitMapping = bm[order, :]
        self.BitsPerSymbol = bm.shape[1]

    def Bit2Symbol(self, BinaryStream):
        b = np.asarray(BinaryStream).reshape(-1)
        m = self.BitsPerSymbol
        idx = _bi2de(b.reshape(-1, m))
        return self.SymbolMapping[idx]

    def _nearest(self, x):
        x = _col(x)
        d = np.abs(x[:, None] - self.SymbolMapping[None, :])
        return np.argmin(d, axis=1)            # first minimum wins, SignalConstellation.m:88

    def Symbol2Bit(self, EstimatedDataSymbols):
        return self.BitMapping[self._nearest(EstimatedDataSymbols), :].reshape(-1).astype(np.uint8)

    def SymbolQuantization(self, EstimatedDataSymbols):
        return self.SymbolMapping[self._nearest(EstimatedDataSymbols)]
