#!/usr/bin/env python3
"""Generates the committed golden fixtures of tests/golden/.

* philox_kat.json     — Random123 known-answer vectors of Philox4x32-10
                        (published with Random123's kat_vectors; copied as data).
* theory_4qam.json    — the reference's own closed form of the 4-QAM doubly-flat
                        Rayleigh BEP, SimpleVersion_DoublyFlat.m:179:
                        BEP = 1/2 - 1/(2 sqrt(2 (1 + 10^(-SNR/10)) - 1)).
* oracle_c2_small.json — regression vectors of the CPU oracle (this repo's
                        restatement, NOT reference output): C2 OFDM, seed
                        0x5EED0002, realisations 0..1, all 7 SNR points —
                        IR samples, R_hP diagonal, error counts.  Parity of the
                        GPU engine is checked against the live oracle; this file
                        pins the oracle against silent drift.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "channel-estimation_amd"), os.path.join(ROOT, "tests")]


def main():
    kat = [
        {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
        {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2, "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
        {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
         "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
    ]
    json.dump(kat, open(os.path.join(HERE, "philox_kat.json"), "w"), indent=1)
    snr = list(range(0, 41, 5))
    bep = [0.5 - 1.0 / (2.0 * np.sqrt(2.0 * (1.0 + 10.0 ** (-s / 10.0)) - 1.0)) for s in snr]
    json.dump({"snr_db": snr, "bep": bep, "source": "SimpleVersion_DoublyFlat.m:179"},
              open(os.path.join(HERE, "theory_4qam.json"), "w"), indent=1)

    import harness
    from dsce.configs import build_setup
    from oracle import refsim
    S = build_setup("default", schemes=("ofdm",))
    sc = S.schemes["ofdm"]
    mm = harness.oracle_mmse(S, sc)
    seed = 0x5EED0002
    tr = {}
    res = refsim.simulate(seed, 0, 2, harness.oracle_chan(S), [harness.oracle_scheme(sc)], S.pn_time, S.n_iter,
                          [mm], trace=tr)
    ir = tr["ir"][0]
    out = {"seed": seed, "reps": [0, 2], "config": "C2 ofdm",
           "ir_rep0_samples": {str(n): [ir[n, 0].real, ir[n, 0].imag, ir[n, 1].real, ir[n, 1].imag]
                               for n in (0, 1, 100, 539)},
           "rhp_diag": [[z.real, z.imag] for z in np.diag(mm["R_hP"])],
           "err": res["err"].tolist(), "nbits": res["nbits"].tolist()}
    json.dump(out, open(os.path.join(HERE, "oracle_c2_small.json"), "w"))
    print("golden fixtures written")


if __name__ == "__main__":
    main()
