"""The Monte-Carlo loop of ``SimpleVersion_DoublyFlat.m`` (BASELINE config 1)
on the HIP engine.

The script (:89-176) draws every random quantity of a realisation — bits,
pilots, the flat channel h and the noise — inside its SNR loop, so each
(realisation, SNR point) is independent.  The engine runs one SNR point per
``dsce_run`` with the Philox key ``snr_seed(seed, k)``; inside that run the
streams follow include/dsce.h (h: THETA stream of the time-invariant
FastFading, noise slot 0 = n_FBMC, slot 1 = n_OFDM).  The one-tap estimate of
each scheme is the PSACE 'linear' interpolation (:143-145) given to the engine
as its weight matrix (dsce_set_interpolation); there are no IC iterations.

Curves (script :164-169, plotted at :186-192):
  FBMC auxiliary, FBMC coding, OFDM (interpolated channel) and FBMC coding /
  OFDM with perfect channel knowledge.
"""
from __future__ import annotations

import numpy as np

from .configs import build_doubly_flat_setup
from .engine import Engine

SCHEMES = ("fbmc_aux", "fbmc_cod", "ofdm")
MASK64 = (1 << 64) - 1


def snr_seed(seed, k):
    """Philox key of SNR point k: seed + k * 2^32 (mod 2^64)."""
    return (int(seed) + (int(k) << 32)) & MASK64


class DoublyFlatSim:
    """Engine configured like SimpleVersion_DoublyFlat.m:16-82."""

    def __init__(self, setup=None, device=0, batch=None):
        self.setup = setup or build_doubly_flat_setup()
        S = self.setup
        eng = Engine(device)
        eng.set_channel(S.channel)
        eng.set_snr(S.pn_time[:1], 0)
        self.sid = {}
        for name in SCHEMES:
            sc = S.schemes[name]
            sid = eng.add_scheme(sc)
            eng.set_noise_slot(sid, sc.extras["noise_slot"])
            eng.set_interpolation(sid, sc.extras["interp"])
            self.sid[name] = sid
        if batch:
            eng.set_batch(batch)
        self.engine = eng

    def run(self, seed, first_rep, n_rep):
        """Bit-error counts int64[scheme, csi (0 interpolated, 1 perfect), snr]
        over realisations [first_rep, first_rep + n_rep)."""
        S = self.setup
        out = np.zeros((len(SCHEMES), 2, len(S.pn_time)), dtype=np.int64)
        for k, pn in enumerate(S.pn_time):
            self.engine.set_snr(np.array([pn]), 0)
            c = self.engine.run(snr_seed(seed, k), first_rep, n_rep)
            out[:, :, k] = c[:, :, 0, 0, 0]
        return out

    def bits_per_rep(self):
        return np.array([self.engine.bits_per_rep(self.sid[n])[0] for n in SCHEMES], dtype=np.int64)

    def ber(self, counts, n_rep):
        """The script's five curves, mean over realisations (:186-191)."""
        b = self.bits_per_rep()[:, None] * n_rep
        return {
            "FBMC Auxiliary": counts[0, 0] / b[0],
            "FBMC Coding": counts[1, 0] / b[1],
            "OFDM": counts[2, 0] / b[2],
            "FBMC perfect CSI": counts[1, 1] / b[1],
            "OFDM perfect CSI": counts[2, 1] / b[2],
        }

    def close(self):
        self.engine.close()
