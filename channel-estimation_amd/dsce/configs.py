"""Experiment setup of ``DoublySelectiveChannelEstimation.m`` (script:16-205).

``build_setup(name)`` reproduces the script's parameter block and object
construction for the BASELINE.json configurations and returns, per
transmission scheme, the operator bundle that crosses the C-ABI:

* G (N x LK) and Q (N x LK) with ``y = Q' r`` (script:191-195),
* the precoder P (LK x Nsym) with ``x = P [xP; xD]`` (script:371-373),
* pilot / data positions, kappa, data-power reduction, the detection rule and
  the no-edge masks (script:131-172).

Names: C2 = 'ofdm24x14' (OFDM 24 sc x 14 sym), C3/C4 = FBMC auxiliary /
data-spreading 24 x 30, C5 = 48 x 30 at SR = 720 kHz (build-defined, SURVEY §7
hard part 8), 'paper' = script:42-46 uncommented.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .channel import FastFading
from .estimation import ImaginaryInterferenceCancellationAtPilotPosition as IIC
from .modulation import FBMC, OFDM, SignalConstellation, mround


def _col(x):
    return np.asarray(x).reshape(-1, order="F")


@dataclass
class Scheme:
    """Everything one transmission scheme hands to the engine."""
    name: str
    kind: str                       # 'ofdm' | 'fbmc_aux' | 'fbmc_cod'
    G: np.ndarray                   # N x LK complex
    Q: np.ndarray                   # N x LK complex, y = Q^H r
    P: np.ndarray                   # LK x Nsym complex
    pilot_pos: np.ndarray           # (NP,) positions in LK (0-based, column-major)
    data_pos: np.ndarray            # (ND,) positions in LK used for detection ('select' mode)
    despread: bool                  # True: x = P^H (y ./ h), take entries NP.. (script:436-437)
    real_detect: bool               # FBMC: real() before detection
    data_div: float                 # divisor applied before detection
    kappa: float
    dpr: float
    const: SignalConstellation      # data constellation (PAM-16 for FBMC, QAM-256 for OFDM)
    considered_symbols: np.ndarray  # (ND,) bool no-edge mask per data symbol
    n_pilots: int
    n_data: int
    bits_slot: int = 0              # RNG sub-stream of the data bits (script:355-357 draw order)
    pilot_slot: int = 0             # RNG sub-stream of the pilots; FBMC aux/cod share xP (script:365)
    extras: dict = field(default_factory=dict)

    @property
    def LK(self):
        return self.G.shape[1]

    @property
    def bits_per_symbol(self):
        return self.const.BitsPerSymbol

    @property
    def n_bits(self):
        return self.n_data * self.bits_per_symbol


@dataclass
class Setup:
    name: str
    N: int
    L: int
    F: float
    SR: float
    snr_db: np.ndarray
    pn_time: np.ndarray             # noise power per SNR (script:243 / :398)
    n_iter: int
    zero_threshold: float
    channel: FastFading
    schemes: dict
    n_repetitions: int
    plot_snr_db: float


_CONFIGS = {
    # script:18-37 (default block)
    "default": dict(L=24, SRmul=24, subframes=1, snr=np.arange(10, 41, 5), reps=25, plot=35),
    # 48 subcarriers: SR = F*48 so that SR >= L*F (FBMC.m:77-79); SURVEY §7 hard part 8
    "c5": dict(L=48, SRmul=48, subframes=1, snr=np.arange(10, 41, 2), reps=10000, plot=32),
    # script:42-46 uncommented (the paper)
    "paper": dict(L=24, SRmul=14 * 14, subframes=2, snr=np.arange(10, 41, 2), reps=1000, plot=32),
}

ALIASES = {"ofdm24x14": "default", "c2": "default", "c3": "default", "c4": "default",
           "fbmc_aux24x30": "default", "fbmc_cod24x30": "default", "c5": "c5", "paper": "paper",
           "default": "default"}


def build_setup(name="default", schemes=("fbmc_aux", "fbmc_cod", "ofdm"), snr_db=None, n_iter=4, tx=None):
    """The script's setup (script:16-205).  ``tx``: optional producer of
    (G, Q = GetRXMatrix') for a modulation object, e.g. dsce.engine.gpu_tx
    (dsce_tx_matrices, row f1: G and Q in closed form on the GPU instead of
    L K Modulation() calls); default: the host mirror's GetTXMatrix /
    GetRXMatrix."""
    cfg = _CONFIGS[ALIASES[name]]

    def txrx(mod):
        if tx is not None:
            return tx(mod)
        return mod.GetTXMatrix(), mod.GetRXMatrix().conj().T
    L = cfg["L"]
    F = 15e3
    SR = F * cfg["SRmul"]
    nsub = cfg["subframes"]
    qam_order = 256
    p2d = 2.0
    p2d_aux = 4.685
    velocity = 500.0
    snr = np.asarray(cfg["snr"] if snr_db is None else snr_db, dtype=float)

    fbmc = FBMC(L, 30 * nsub, F, SR, 0, False, "Hermite-OQAM", 8, 0, True)
    zg_time = ((fbmc.Nr.SamplesTotal - (mround((1 / 15e3 / 14) * SR) + mround(SR / 15e3)) * 14 * nsub) / 2) / SR
    ofdm = OFDM(L, 14 * nsub, F, SR, 0, False, 1 / 15e3 / 14, zg_time)
    if ofdm.Nr.SamplesTotal != fbmc.Nr.SamplesTotal:
        raise ValueError("Total number of samples must be the same for OFDM and FBMC.")
    N = ofdm.Nr.SamplesTotal

    pam = SignalConstellation(int(np.sqrt(qam_order)), "PAM")
    qam = SignalConstellation(qam_order, "QAM")

    # pilot matrices, script:91-103 (1-based MATLAB ranges -> 0-based)
    pm_ofdm = np.zeros((L, 14))
    pm_ofdm[1::12, 1::7] = 1
    pm_ofdm[4::12, 5::7] = 1
    pm_ofdm[7::12, 1::7] = 1
    pm_ofdm[10::12, 5::7] = 1
    pm_ofdm = np.tile(pm_ofdm, (1, nsub))
    pm_fbmc = np.zeros((L, 30))
    pm_fbmc[1::12, 2::16] = 1
    pm_fbmc[4::12, 10::16] = 1
    pm_fbmc[7::12, 3::16] = 1
    pm_fbmc[10::12, 11::16] = 1
    pm_fbmc = np.tile(pm_fbmc, (1, nsub))

    aux_pm = pm_fbmc.copy()                                    # script:106-113
    a, b = np.nonzero(pm_fbmc.T)
    a, b = b, a                                                # MATLAB find order (column-major)
    for l, k in zip(a, b):
        aux_pm[l + 1, k] = -1
        aux_pm[l - 1, k] = -1
        aux_pm[l, k + 1] = -1
        aux_pm[l, k - 1] = -1

    NP = int(np.sum(pm_ofdm == 1))                             # script:131
    ND_ofdm = int(np.sum(pm_ofdm == 0))
    LK_ofdm = pm_ofdm.size

    # edge masks, script:145-149
    cons_fbmc = np.zeros(pm_fbmc.shape)
    cons_fbmc[4:pm_fbmc.shape[0] - 4, 10:pm_fbmc.shape[1] - 10] = 1
    cons_ofdm = np.zeros(pm_ofdm.shape)
    cons_ofdm[4:pm_ofdm.shape[0] - 4, 5:pm_ofdm.shape[1] - 5] = 1

    out = {}
    need_fbmc = any(s.startswith("fbmc") for s in schemes)
    if need_fbmc:
        G_fbmc, Q_fbmc = txrx(fbmc)                            # script:191-192
        Dfbmc = fbmc.GetFBMCMatrix()
    if "fbmc_aux" in schemes:
        aux = IIC("Auxiliary", aux_pm, Dfbmc, 28, p2d_aux)     # script:116-122
        kappa = aux.PilotToDataPowerOffset * aux.DataPowerReduction
        nd = aux.NrDataSymbols
        cm = np.zeros(nd, dtype=bool)                          # script:151-156
        sel = (_col(cons_fbmc) * (_col(aux_pm) == 0)) == 1
        eye_nd = np.eye(nd)
        xs = aux.PrecodingMatrix[:, NP:]                        # P * [0; e_i] = column NP+i
        for i in range(nd):
            cm[i] = np.sum(np.abs(xs[sel, i])) > aux.DataPowerReduction * 0.9
        del eye_nd
        out["fbmc_aux"] = Scheme(
            name="fbmc_aux", kind="fbmc_aux", G=G_fbmc, Q=Q_fbmc, P=aux.PrecodingMatrix,
            pilot_pos=np.flatnonzero(_col(pm_fbmc) == 1), data_pos=np.flatnonzero(_col(aux_pm) == 0),
            despread=False, real_detect=True, data_div=float(np.sqrt(aux.DataPowerReduction)),
            kappa=float(kappa), dpr=aux.DataPowerReduction, const=pam, considered_symbols=cm,
            n_pilots=NP, n_data=nd, bits_slot=0, pilot_slot=0, extras=dict(iic=aux, pilot_matrix=aux_pm, modulation=fbmc))
    if "fbmc_cod" in schemes:
        cod = IIC("Coding", pm_fbmc, Dfbmc, 20, 2 * p2d)        # script:123-129
        kappa = cod.PilotToDataPowerOffset * cod.DataPowerReduction
        nd = cod.NrDataSymbols
        notcons = _col(cons_fbmc) == 0
        xs = cod.PrecodingMatrix[:, NP:]
        cm = ~np.any(xs[notcons, :] != 0, axis=0)              # script:157-162
        out["fbmc_cod"] = Scheme(
            name="fbmc_cod", kind="fbmc_cod", G=G_fbmc, Q=Q_fbmc, P=cod.PrecodingMatrix,
            pilot_pos=np.flatnonzero(_col(pm_fbmc) == 1), data_pos=np.arange(NP, cod.PrecodingMatrix.shape[1]),
            despread=True, real_detect=True, data_div=float(cod.DataPowerReduction),
            kappa=float(kappa), dpr=cod.DataPowerReduction, const=pam, considered_symbols=cm,
            n_pilots=NP, n_data=nd, bits_slot=1, pilot_slot=0, extras=dict(iic=cod, pilot_matrix=pm_fbmc, modulation=fbmc))
    if "ofdm" in schemes:
        G_ofdm, Q_ofdm = txrx(ofdm)                            # script:194-195
        pmv = _col(pm_ofdm)
        PMap = np.zeros((LK_ofdm, LK_ofdm))                    # script:134-137
        PMap[np.ix_(pmv == 1, np.arange(NP))] = np.sqrt(p2d) * np.eye(NP)
        PMap[np.ix_(pmv == 0, np.arange(NP, LK_ofdm))] = np.eye(ND_ofdm)
        PMap = PMap / np.sqrt(np.mean(np.diag(PMap @ PMap.T)))
        dpr = LK_ofdm / (NP * p2d + ND_ofdm)                   # script:138
        kappa = p2d * dpr                                       # script:142
        sel = (_col(cons_ofdm) * (pmv == 0)) == 1
        xs = PMap[:, NP:]
        cm = np.array([np.sum(np.abs(xs[sel, i])) > dpr * 0.9 for i in range(ND_ofdm)])
        out["ofdm"] = Scheme(
            name="ofdm", kind="ofdm", G=G_ofdm, Q=Q_ofdm, P=PMap.astype(complex),
            pilot_pos=np.flatnonzero(pmv == 1), data_pos=np.flatnonzero(pmv == 0),
            despread=False, real_detect=False, data_div=float(np.sqrt(dpr)),
            kappa=float(kappa), dpr=float(dpr), const=qam, considered_symbols=cm,
            n_pilots=NP, n_data=ND_ofdm, bits_slot=2, pilot_slot=1, extras=dict(pilot_matrix=pm_ofdm, ofdm=ofdm, modulation=ofdm))

    fD = velocity / 3.6 * 2.5e9 / 2.998e8                      # script:180
    chan = FastFading(SR, "VehicularA", N, fD, "Jakes", 200, 1, 1, 1)
    pn = SR / (F * L) * 10.0 ** (-snr / 10)                    # script:243 / :398
    return Setup(name=name, N=N, L=L, F=F, SR=SR, snr_db=snr, pn_time=pn, n_iter=n_iter,
                 zero_threshold=1e-8, channel=chan, schemes=out, n_repetitions=cfg["reps"],
                 plot_snr_db=cfg["plot"])


# ---------------------------------------------------------------------------
# SimpleVersion_DoublyFlat.m (BASELINE config 1): doubly-flat channel, pilot
# interpolation instead of the MMSE estimator, no interference cancellation.
# ---------------------------------------------------------------------------
def build_doubly_flat_setup(qam_order=16, snr_db=None, n_repetitions=1000, interpolation="linear", block=None):
    """Setup of ``SimpleVersion_DoublyFlat.m`` (:12-82).

    Schemes 'fbmc_aux', 'fbmc_cod', 'ofdm' with their interpolation weights
    (``extras['interp']``, PSACE 'linear' on the Diamond patterns, :47-66) and
    noise slots (``extras['noise_slot']``: n_FBMC shared by the two FBMC
    schemes, n_OFDM separate, :125-126).  The channel is the time-invariant
    'Flat' FastFading (fD = 0, FastFading.m:241-246), i.e. the script's
    h = sqrt(1/2) (randn + j randn) (:123).  The script draws everything —
    bits, pilots, h, noise — inside its SNR loop (:90-126); the engine runs one
    SNR point per call with the key ``snr_seed(seed, k)`` (dsce.doubly_flat).
    ``interpolation`` selects the PSACE method (the script uses 'linear';
    'nearest', 'natural', 'FullAverage' and 'MovingBlockAverage' with ``block``
    = [BlockLengthFrequency, BlockLengthTime] are the class's other methods,
    PSACE.m:73-99): all are linear in the LS estimates, so each crosses the ABI
    as one weight matrix.
    """
    from .estimation import PilotSymbolAidedChannelEstimation as PSACE
    L = 12
    F = 15e3
    SR = 15e3 * 14 * 12
    snr = np.asarray(np.arange(0, 31, 5) if snr_db is None else snr_db, dtype=float)
    fbmc = FBMC(L, 30, F, SR, 15e3 * 20, False, "Hermite-OQAM", 8, 0, True)          # :17-28
    ofdm = OFDM(L, 15, F, SR, 15e3 * 20, False, 0, (8 - 1 / 2) * 1 / 15e3 * 1 / 2)   # :31-40
    N = ofdm.Nr.SamplesTotal
    if fbmc.Nr.SamplesTotal != N:
        raise ValueError("Total number of samples must be the same for OFDM and FBMC.")
    pam = SignalConstellation(int(np.sqrt(qam_order)), "PAM")                       # :43-44
    qam = SignalConstellation(qam_order, "QAM")
    ce_ofdm = PSACE("Diamond", [[ofdm.Nr.Subcarriers, 6], [ofdm.Nr.MCSymbols, 4]], interpolation, block)   # :47-56
    ce_fbmc = PSACE("Diamond", [[fbmc.Nr.Subcarriers, 6], [fbmc.Nr.MCSymbols, 8]], interpolation, block)   # :57-66
    Dfbmc = fbmc.GetFBMCMatrix()
    aux_pm = ce_fbmc.GetAuxiliaryMatrix(1)
    aux = IIC("Auxiliary", aux_pm, Dfbmc, 16, 2)                                      # :69-75
    cod = IIC("Coding", ce_fbmc.PilotMatrix, Dfbmc, 16, 2)                            # :76-82
    G_fbmc = fbmc.GetTXMatrix()
    Q_fbmc = fbmc.GetRXMatrix().conj().T
    G_ofdm = ofdm.GetTXMatrix()
    Q_ofdm = ofdm.GetRXMatrix().conj().T
    W_fbmc = ce_fbmc.GetInterpolationWeights()
    W_ofdm = ce_ofdm.GetInterpolationWeights()
    NPf = ce_fbmc.NrPilotSymbols
    pil_f = np.flatnonzero(_col(ce_fbmc.PilotMatrix) == 1)
    out = {}
    out["fbmc_aux"] = Scheme(                                                         # :138, :148, :156
        name="fbmc_aux", kind="fbmc_aux", G=G_fbmc, Q=Q_fbmc, P=aux.PrecodingMatrix, pilot_pos=pil_f,
        data_pos=np.flatnonzero(_col(aux.PilotMatrix) == 0), despread=False, real_detect=True,
        data_div=float(np.sqrt(aux.DataPowerReduction)),
        kappa=float(aux.PilotToDataPowerOffset * aux.DataPowerReduction), dpr=aux.DataPowerReduction, const=pam,
        considered_symbols=np.ones(aux.NrDataSymbols, dtype=bool), n_pilots=NPf, n_data=aux.NrDataSymbols,
        bits_slot=0, pilot_slot=0,
        extras=dict(iic=aux, pilot_matrix=aux_pm, modulation=fbmc, interp=W_fbmc, noise_slot=0, psace=ce_fbmc))
    out["fbmc_cod"] = Scheme(                                                         # :139, :149-150, :157-158
        name="fbmc_cod", kind="fbmc_cod", G=G_fbmc, Q=Q_fbmc, P=cod.PrecodingMatrix, pilot_pos=pil_f,
        data_pos=np.arange(NPf, cod.PrecodingMatrix.shape[1]), despread=True, real_detect=True, data_div=1.0,
        kappa=float(cod.PilotToDataPowerOffset), dpr=cod.DataPowerReduction, const=pam,
        considered_symbols=np.ones(cod.NrDataSymbols, dtype=bool), n_pilots=NPf, n_data=cod.NrDataSymbols,
        bits_slot=1, pilot_slot=0,
        extras=dict(iic=cod, pilot_matrix=ce_fbmc.PilotMatrix, modulation=fbmc, interp=W_fbmc, noise_slot=0,
                    psace=ce_fbmc))
    pmv = _col(ce_ofdm.PilotMatrix)
    NPo = ce_ofdm.NrPilotSymbols
    LKo = pmv.size
    Pm = np.zeros((LKo, LKo))                                                          # :113-115
    Pm[np.flatnonzero(pmv == 1), np.arange(NPo)] = 1.0
    Pm[np.flatnonzero(pmv == 0), np.arange(NPo, LKo)] = 1.0
    out["ofdm"] = Scheme(                                                             # :140, :152-153, :160-161
        name="ofdm", kind="ofdm", G=G_ofdm, Q=Q_ofdm, P=Pm.astype(complex), pilot_pos=np.flatnonzero(pmv == 1),
        data_pos=np.flatnonzero(pmv == 0), despread=False, real_detect=False, data_div=1.0, kappa=1.0, dpr=1.0,
        const=qam, considered_symbols=np.ones(LKo - NPo, dtype=bool), n_pilots=NPo, n_data=LKo - NPo,
        bits_slot=2, pilot_slot=1,
        extras=dict(pilot_matrix=ce_ofdm.PilotMatrix, modulation=ofdm, interp=W_ofdm, noise_slot=1, psace=ce_ofdm))
    chan = FastFading(SR, "Flat", N, 0.0, "Jakes", 1, 1, 1, 0)
    pn = SR / (F * L) * 10.0 ** (-snr / 10)                                            # :92
    return Setup(name="doubly_flat", N=N, L=L, F=F, SR=SR, snr_db=snr, pn_time=pn, n_iter=0, zero_threshold=1e-8,
                 channel=chan, schemes=out, n_repetitions=n_repetitions, plot_snr_db=float(snr[-1]))
