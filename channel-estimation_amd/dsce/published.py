"""BER points of the reference's published figures (png/Figure3.png,
png/Figure5.png, README.md:26,30), digitised from the plot frames (log axis,
about +-3 %).  Paper configuration = script:42-46 uncommented:
FBMC-OQAM with 4 auxiliary symbols per pilot, 24 x 60, SR = 196 F, N = 7350,
VehicularA at 500 km/h and 2.5 GHz, 16 SNR points 10:2:40 dB, 4 IC iterations.

Keys index the engine's counter array of one scheme: (csi, edge, stage) with
csi 0 = MMSE estimate, 1 = perfect CSI; edge 0 = all bits, 1 = no-edge bits;
stage 0 = one-tap, i = IC iteration i."""

FIGURE3 = {
    "one-tap MMSE": ((0, 0, 0), {10: 0.286, 20: 0.141, 30: 0.0796, 32: 0.0751, 40: 0.0678}),
    "one-tap perfect CSI": ((1, 0, 0), {10: 0.277, 30: 0.0714, 32: 0.0674, 40: 0.0615}),
    "IC4 MMSE": ((0, 0, 4), {10: 0.280, 30: 0.0297, 32: 0.0218, 36: 0.0128}),
    "IC4 MMSE no edges": ((0, 1, 4), {10: 0.280, 20: 0.115, 30: 0.0268, 32: 0.0188, 36: 0.0105}),
    "IC4 perfect CSI": ((1, 0, 4), {10: 0.280, 20: 0.110, 30: 0.0223, 32: 0.0159, 34: 0.0118}),
}

# BER vs IC iteration (stage 0..4) at 32 dB
FIGURE5_32DB = {
    "MMSE": ((0, 0), [0.0747, 0.0298, 0.0236, 0.0224, 0.0217]),
    "MMSE no edges": ((0, 1), [0.0730, 0.0258, 0.0203, 0.0193, 0.0188]),
    "perfect CSI": ((1, 0), [0.0676, 0.0211, 0.0170, 0.0162, 0.0158]),
}


def compare(ber, snr_db):
    """Rows {curve, snr_db, [stage], ber, published, ratio} for a BER array
    ber[csi][edge][snr][stage] of the auxiliary-symbol scheme."""
    snr = [float(x) for x in snr_db]
    rows = []
    for name, ((csi, edge, st), pts) in FIGURE3.items():
        for s, ref in pts.items():
            b = float(ber[csi][edge][snr.index(float(s))][st])
            rows.append({"curve": "Fig3 " + name, "snr_db": s, "ber": b, "published": ref, "ratio": b / ref})
    k32 = snr.index(32.0)
    for name, ((csi, edge), pts) in FIGURE5_32DB.items():
        for st, ref in enumerate(pts):
            b = float(ber[csi][edge][k32][st])
            rows.append({"curve": "Fig5 " + name, "snr_db": 32, "stage": st, "ber": b, "published": ref,
                         "ratio": b / ref})
    return rows
