"""GPU: the C-ABI's host code under AddressSanitizer ("race
detection / sanitizers"; host code only: GPU ASAN is not available on the
pool).  `make -f asan.mk` (run by __graft_entry__.build) compiles dsce_api.hip with
-fsanitize=address on the host side and links it with the regular kernel
objects into tools/asan/dsce_asan_driver.  The driver replays the MATLAB
host's call sequence from a setup dump, on a
single-device context and on a two-member multi-device context (member
threads, host sum), plus the boundary's error paths, and compares the counts
with the regular library's for the same inputs.  It runs as its own process,
so no sanitizer runtime enters the Python interpreter."""
import os
import subprocess

import numpy as np
import pytest

import harness

pytestmark = pytest.mark.gpu

BIN = os.path.join(harness.ROOT, "tools", "asan", "dsce_asan_driver")
SEED, FIRST, NREP, BATCH = 0x5EED0003, 7, 300, 128
MODELS = {"Jakes": 0, "Uniform": 1, "Discrete-Jakes": 2, "Discrete-Uniform": 3}


def _cplx(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.complex128).reshape(-1, order="F")).view(np.float64)


def _dump(path, S, sc, expect):
    """The driver's input, in the order asan_driver.cpp reads it; the arrays are
    the ones dsce.engine.Engine.set_channel / add_scheme hand to the ABI."""
    ch = S.chan
    pdp = np.asarray(ch["pdp_norm"], dtype=np.float64)
    pn = np.asarray(S.pn_time, dtype=np.float64)
    L = sc.extras["pilot_matrix"].shape[0] if "pilot_matrix" in sc.extras else sc.LK
    parts = [
        np.array([S.N, pdp.size, ch["paths"], MODELS[ch["model"]], pn.size, S.n_iter, BATCH, 0], dtype=np.int32),
        np.array([1.0 / ch["dt"], ch["fD"], S.zero_threshold], dtype=np.float64),
        pdp, pn,
        np.array([L, sc.LK // L, sc.P.shape[1], sc.n_pilots, sc.n_data, sc.const.ModulationOrder,
                  sc.bits_per_symbol, int(sc.despread), int(sc.real_detect), sc.bits_slot, sc.pilot_slot],
                 dtype=np.int32),
        np.array([sc.kappa, sc.data_div], dtype=np.float64),
        _cplx(sc.G), _cplx(sc.Q), _cplx(sc.P),
        np.asarray(sc.pilot_pos, dtype=np.int32), np.asarray(sc.data_pos, dtype=np.int32),
        np.asarray(sc.considered_symbols, dtype=np.uint8), _cplx(sc.const.SymbolMapping),
        np.array([SEED, FIRST, NREP], dtype=np.uint64),
        np.ascontiguousarray(expect, dtype=np.int64).ravel(),
    ]
    with open(path, "wb") as f:
        for p in parts:
            f.write(np.ascontiguousarray(p).tobytes())


def test_c_abi_under_host_asan(tmp_path):
    assert os.path.exists(BIN), "tools/asan/dsce_asan_driver missing: run __graft_entry__.build() (make -f asan.mk)"
    S = harness.setup("default", schemes=("ofdm",))
    eng = harness.engine(S, batch=BATCH)
    try:
        expect = eng.run(SEED, FIRST, NREP)
    finally:
        eng.close()
    assert expect.sum() > 0
    dump = str(tmp_path / "setup.bin")
    _dump(dump, S, harness._engine_scheme(S, "ofdm"), expect)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0")
    r = subprocess.run([BIN, dump], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan driver: 0 failure(s)" in r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr
    # and the sanitizer is live in this binary: a deliberate overflow is caught
    p = subprocess.run([BIN, "--probe"], env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "heap-buffer-overflow" in p.stderr, p.stderr[-2000:]
