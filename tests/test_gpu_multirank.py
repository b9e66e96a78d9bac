"""GPU, multi-rank: `dsce.simulate` sharded over 2 ranks (one process per GPU
in production with RCCL; here both ranks share the box's one GPU over gloo,
DSCE_DIST_BACKEND=gloo) gives exactly the counters and MSE sums of a single
rank over the same realisations — the contiguous realisation shards plus one
all-reduce of SURVEY §8e."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import harness

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_simulate_two_ranks_equals_one(tmp_path):
    args = ["--config", "default", "--schemes", "ofdm,fbmc_aux", "--reps", "1024", "--batch", "256", "--mse"]
    env = dict(os.environ, DSCE_DIST_BACKEND="gloo", PYTHONPATH=harness.PKG)
    one = tmp_path / "one.json"
    two = tmp_path / "two.json"
    subprocess.run([sys.executable, "-m", "dsce.simulate", *args, "--out", str(one)], cwd=harness.PKG, env=env,
                   check=True, timeout=240, capture_output=True)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "dsce.simulate", *args,
                    "--out", str(two)], cwd=harness.PKG, env=env, check=True, timeout=240, capture_output=True)
    a, b = json.load(open(one)), json.load(open(two))
    assert b["ranks"] == 2 and a["ranks"] == 1
    assert np.array_equal(np.array(a["counts"]), np.array(b["counts"]))
    for s in ("ofdm", "fbmc_aux"):
        np.testing.assert_allclose(np.array(a["nmse"][s]), np.array(b["nmse"][s]), rtol=1e-12)


def test_simulate_snr_shards_equal_one_rank(tmp_path):
    """--shard snr: 2 ranks take 4 + 3 of the 7 SNR points, each with only its own
    estimator (snr_base keys the noise by the sweep's SNR index); counters and
    MSE sums equal the one-rank run exactly.  An odd realisation count
    (64 x 5) is not padded to a multiple of 64 x world."""
    args = ["--config", "default", "--schemes", "ofdm,fbmc_aux", "--reps", "320", "--batch", "128", "--mse"]
    env = dict(os.environ, DSCE_DIST_BACKEND="gloo", PYTHONPATH=harness.PKG)
    one, two, three = tmp_path / "one.json", tmp_path / "two.json", tmp_path / "three.json"
    subprocess.run([sys.executable, "-m", "dsce.simulate", *args, "--out", str(one)], cwd=harness.PKG, env=env,
                   check=True, timeout=240, capture_output=True)
    for nproc, out, shard in ((2, two, "snr"), (3, three, "reps")):
        subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "dsce.simulate", *args,
                        "--shard", shard, "--out", str(out)], cwd=harness.PKG, env=env, check=True, timeout=300,
                       capture_output=True)
    a = json.load(open(one))
    for f in (two, three):
        b = json.load(open(f))
        assert b["n_repetitions"] == a["n_repetitions"] == 320
        assert np.array_equal(np.array(a["counts"]), np.array(b["counts"]))
        for s in ("ofdm", "fbmc_aux"):
            np.testing.assert_allclose(np.array(a["nmse"][s]), np.array(b["nmse"][s]), rtol=1e-12)


def test_bench_gpus_flag_launches_ranks():
    """bench.py --gpus 2 without a launcher starts torch.distributed.run itself
    (one rank per GPU; here both ranks share the one GPU over gloo) and forwards
    rank 0's JSON line, which reports both ranks' realisations."""
    env = dict(os.environ, DSCE_DIST_BACKEND="gloo")
    out = subprocess.run([sys.executable, os.path.join(harness.ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "1", "--reps-per-step", "1024", "--no-cpu-baseline"], env=env, check=True,
                         timeout=300, capture_output=True, text=True)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["value"] > 0
    bad = subprocess.run([sys.executable, os.path.join(harness.ROOT, "bench.py"), "--gpus", "2"],
                         env=dict(env, WORLD_SIZE="1"), timeout=120, capture_output=True, text=True)
    assert bad.returncode != 0


def test_rccl_allreduce_one_rank(tmp_path):
    """The counter all-reduce on the RCCL path (backend 'nccl' = RCCL on ROCm,
    device tensors), exercised on the one-GPU box: dsce.simulate under
    torch.distributed.run --nproc-per-node 1 with the default backend reports an
    all-reduce over nccl on a cuda tensor and returns exactly the counts and the MSE
    sums of the plain single-process run.  The same code path carries the 8-rank
    run of SURVEY §8e; only the world size differs.  (The MSE sums are fp64
    atomics whose order varies between runs: equal to 1e-12.)"""
    args = ["--config", "default", "--schemes", "ofdm", "--reps", "512", "--batch", "256", "--mse"]
    env = {k: v for k, v in os.environ.items() if k != "DSCE_DIST_BACKEND"}
    env["PYTHONPATH"] = harness.PKG
    one, ranked = tmp_path / "one.json", tmp_path / "rccl.json"
    subprocess.run([sys.executable, "-m", "dsce.simulate", *args, "--out", str(one)], cwd=harness.PKG, env=env,
                   check=True, timeout=240, capture_output=True)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                    "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "dsce.simulate", *args,
                    "--out", str(ranked)], cwd=harness.PKG, env=env, check=True, timeout=240, capture_output=True)
    a, b = json.load(open(one)), json.load(open(ranked))
    ar = b["allreduce"]
    assert ar["backend"] == "nccl" and ar["device"].startswith("cuda") and ar["world"] == 1, ar
    assert "allreduce" not in a
    assert np.array_equal(np.array(a["counts"]), np.array(b["counts"]))
    # the MSE sums are fp64 atomics (their order varies from run to run): rounding level
    np.testing.assert_allclose(np.array(a["nmse"]["ofdm"]), np.array(b["nmse"]["ofdm"]), rtol=1e-12)


def test_eight_rank_control_flow_on_one_gpu(tmp_path):
    """The 8-rank control flow of SURVEY §8e rehearsed on the one-GPU box (8
    gloo ranks share the device): --shard snr over C2's 7
    SNR points leaves rank 7 empty, --shard reps splits an odd 520 realisations
    65 per rank; both equal the one-rank counts and MSE sums.  Then bench.py
    --gpus 8 launches its own ranks and reports the max-over-ranks time."""
    args = ["--config", "default", "--schemes", "ofdm", "--reps", "520", "--batch", "128", "--mse"]
    env = dict(os.environ, DSCE_DIST_BACKEND="gloo", PYTHONPATH=harness.PKG)
    one = tmp_path / "one.json"
    subprocess.run([sys.executable, "-m", "dsce.simulate", *args, "--out", str(one)], cwd=harness.PKG, env=env,
                   check=True, timeout=240, capture_output=True)
    a = json.load(open(one))
    assert len(a["snr_db"]) == 7
    for shard in ("snr", "reps"):
        out = tmp_path / ("eight_%s.json" % shard)
        subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "dsce.simulate", *args,
                        "--shard", shard, "--out", str(out)], cwd=harness.PKG, env=env, check=True, timeout=400,
                       capture_output=True)
        b = json.load(open(out))
        assert b["ranks"] == 8 and b["shard"] == shard and b["n_repetitions"] == 520
        assert np.array_equal(np.array(a["counts"]), np.array(b["counts"])), shard
        np.testing.assert_allclose(np.array(a["nmse"]["ofdm"]), np.array(b["nmse"]["ofdm"]), rtol=1e-12)
    res = subprocess.run([sys.executable, os.path.join(harness.ROOT, "bench.py"), "--gpus", "8", "--steps", "2",
                          "--warmup", "1", "--reps-per-step", "1024", "--no-cpu-baseline"], env=env, check=True,
                         timeout=400, capture_output=True, text=True)
    line = json.loads(res.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 8 and line["config"]["parallelism"] == "dp8"
    assert line["value"] > 0 and line["steps"] == 2


def test_two_ranks_stop_and_resume_from_checkpoints(tmp_path):
    """--checkpoint under a launcher: one file per rank.  With --stop-after 128
    rank 0 (128 realisations) finishes and rank 1 (192) does not, so neither
    rank writes a result (the ranks agree by one all-reduce before the counter
    all-reduce); the resumed launch finishes rank 1 and counts exactly like one
    uninterrupted rank."""
    args = ["--config", "default", "--schemes", "ofdm", "--reps", "320", "--batch", "64", "--mse"]
    env = dict(os.environ, DSCE_DIST_BACKEND="gloo", PYTHONPATH=harness.PKG)
    one, two, ck = tmp_path / "one.json", tmp_path / "two.json", str(tmp_path / "ck.json")
    subprocess.run([sys.executable, "-m", "dsce.simulate", *args, "--out", str(one)], cwd=harness.PKG, env=env,
                   check=True, timeout=240, capture_output=True)
    launch = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1"]
    for extra in (["--stop-after", "128"], ["--resume"]):
        subprocess.run([*launch, "--master-port", str(_port()), "-m", "dsce.simulate", *args, "--checkpoint", ck,
                        "--out", str(two), *extra], cwd=harness.PKG, env=env, check=True, timeout=300,
                       capture_output=True)
        if extra[0] == "--stop-after":
            assert not two.exists()
            assert [json.load(open(ck + ".rank%d" % r))["done"] for r in (0, 1)] == [128, 128]
    a, b = json.load(open(one)), json.load(open(two))
    assert b["ranks"] == 2 and b["resumed"] is True
    assert np.array_equal(np.array(a["counts"]), np.array(b["counts"]))
    np.testing.assert_allclose(np.array(a["nmse"]["ofdm"]), np.array(b["nmse"]["ofdm"]), rtol=1e-12)
