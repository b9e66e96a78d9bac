"""GPU: the multi-device context of the C-ABI (dsce_create_multi, ABI 7) — the
path a MATLAB host (one process, README.md:19-20) uses to shard the
Monte-Carlo loop of DoublySelectiveChannelEstimation.m:350-564 over the GPUs
of a node.  On the one-GPU box:
  * devices [0]: one member, the counters summed by the in-library RCCL
    all-reduce (ncclCommInitAll + ncclAllReduce) — the reduction path of an
    8-GPU node at world size 1;
  * devices [0, 0, 0]: three members on one device (one RCCL rank per device,
    so the counters are summed on the host), exercising the 64-aligned slices
    and the per-member threads.
Both must give the single context's counts bit for bit (the Philox streams are
keyed by the global realisation index) and its MSE sums to rounding (fp64
atomics: order-dependent even between two runs of one context)."""
import numpy as np
import pytest

import harness

pytestmark = pytest.mark.gpu

SEED = 0x5EED0002


@pytest.fixture(scope="module")
def setup_c2():
    return harness.setup("default", schemes=("ofdm",))


@pytest.fixture(scope="module")
def single(setup_c2):
    eng = harness.engine(setup_c2, batch=256)
    eng.enable_mse(True)
    counts = eng.run(SEED, 5, 777)                  # ragged: 12 waves + 9 realisations, odd first_rep
    err, pw = eng.mse()
    eng.close()
    return counts, err, pw


@pytest.mark.parametrize("devices,reduce", [([0], "rccl"), ([0, 0, 0], "host")])
def test_multi_device_counts_equal_single_context(setup_c2, single, devices, reduce):
    eng = harness.engine(setup_c2, batch=256, device=devices)
    try:
        assert eng.group_info() == (devices, reduce)
        eng.enable_mse(True)
        counts = eng.run(SEED, 5, 777)
        err, pw = eng.mse()
        assert eng.path_info(0) >= {"mic_stages", "pic_fft", "txrx_fft"}
    finally:
        eng.close()
    c1, e1, p1 = single
    np.testing.assert_array_equal(counts, c1)
    # the device MSE sums are fp64 atomics (order-dependent rounding, run to run
    # as well): equal to 1e-12 relative
    np.testing.assert_allclose(err, e1, rtol=1e-12, atol=0)
    np.testing.assert_allclose(pw, p1, rtol=1e-12, atol=0)


def test_multi_device_configuration_reaches_every_member(setup_c2):
    """Options and batch reach every member (the shards run the same kernels),
    an empty slice contributes zeros, and counts over a split equal the whole."""
    eng = harness.engine(setup_c2, batch=128, device=[0, 0], options={"mmse_ic": 0})
    try:
        assert eng.get_option("mmse_ic") == 0
        whole = eng.run(SEED, 0, 200)
        assert "mic_stages" not in eng.path_info(0)            # member 0 ran the W contraction
        parts = eng.run(SEED, 0, 64)                             # member 1's slice is empty
        parts = eng.run(SEED, 64, 136, parts)
        np.testing.assert_array_equal(whole, parts)
    finally:
        eng.close()
    ref = harness.engine(setup_c2, batch=128, options={"mmse_ic": 0})
    try:
        np.testing.assert_array_equal(ref.run(SEED, 0, 200), whole)
    finally:
        ref.close()


def test_eight_members_on_one_gpu_rehearse_the_node(setup_c2):
    """The 8-GPU node's control flow on the one-GPU box: eight members (all on
    device 0, so the host sum stands in for the RCCL all-reduce), eight member
    threads, eight 64-aligned slices of an odd realisation count (389 = 6 x 64
    + 5: member 0's slice is empty, member 7's a partial wave), and the
    configuration fanned out to all eight: counts equal the
    single context's over the same realisations."""
    ref = harness.engine(setup_c2, batch=128)
    try:
        want = ref.run(SEED, 3, 389)
    finally:
        ref.close()
    eng = harness.engine(setup_c2, batch=128, device=[0] * 8)
    try:
        assert eng.group_info() == ([0] * 8, "host")
        np.testing.assert_array_equal(eng.run(SEED, 3, 389), want)
    finally:
        eng.close()


def test_multi_device_rejects_bad_devices():
    from dsce.engine import DsceError, Engine
    with pytest.raises(DsceError):
        Engine([0, 4096])
    with pytest.raises(DsceError):
        Engine([])


def test_simulate_devices_flag_equals_one_device(tmp_path):
    """`python -m dsce.simulate --devices ...` (one process, one multi-device
    context: the MATLAB host's path through the Python twin) counts exactly
    like the single-device run, through RCCL ([0]) and the host sum ([0, 0])."""
    import json
    import os
    import subprocess
    import sys
    args = ["--config", "default", "--schemes", "ofdm", "--reps", "300", "--batch", "128"]
    env = dict(os.environ, PYTHONPATH=harness.PKG)
    runs = {}
    for tag, extra in (("one", []), ("rccl", ["--devices", "0"]), ("host", ["--devices", "0,0"])):
        out = tmp_path / (tag + ".json")
        subprocess.run([sys.executable, "-m", "dsce.simulate", *args, *extra, "--out", str(out)], cwd=harness.PKG,
                       env=env, check=True, timeout=240, capture_output=True)
        runs[tag] = json.load(open(out))
    for tag in ("rccl", "host"):
        assert np.array_equal(np.array(runs[tag]["counts"]), np.array(runs["one"]["counts"])), tag
