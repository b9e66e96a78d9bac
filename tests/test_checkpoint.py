"""CPU: the checkpoint file of `python -m dsce.simulate --checkpoint`
(SURVEY section 5 "Checkpoint / resume": the reference has none; with
counter-based streams a resumed run is exact).  The file round-trips the int64
counters and MSE sums, is replaced atomically, and a checkpoint of another run
(other seed, realisation count, shard or rank) is refused rather than mixed in."""
import json
import os

import numpy as np
import pytest

import harness  # noqa: F401  (puts the package on sys.path)
from dsce.simulate import CHECKPOINT_VERSION, load_checkpoint, save_checkpoint

KEY = {"config": "default", "schemes": ["ofdm"], "seed": 7, "reps": 300, "shard": "reps", "world": 1,
       "rank": 0, "first": 0, "mine": 300, "mse": True, "snr": [0, 7]}


def test_round_trip_is_exact(tmp_path):
    p = str(tmp_path / "ck.json")
    rng = np.random.default_rng(1)
    counts = rng.integers(0, 2 ** 62, size=(1, 2, 2, 7, 5), dtype=np.int64)
    err, pw = rng.random((1, 7, 5)), rng.random((1, 7))
    save_checkpoint(p, KEY, 128, counts, 1.5, (err, pw))
    assert not os.path.exists(p + ".tmp")
    d = load_checkpoint(p, dict(KEY))
    assert d["done"] == 128 and d["seconds"] == 1.5 and d["version"] == CHECKPOINT_VERSION
    np.testing.assert_array_equal(np.asarray(d["counts"], dtype=np.int64).reshape(counts.shape), counts)
    np.testing.assert_array_equal(np.asarray(d["mse_err"]).reshape(err.shape), err)   # JSON floats round-trip
    np.testing.assert_array_equal(np.asarray(d["mse_pow"]).reshape(pw.shape), pw)


@pytest.mark.parametrize("field,value", [("seed", 8), ("reps", 301), ("rank", 1), ("shard", "snr"),
                                         ("schemes", ["fbmc_aux"]), ("mse", False)])
def test_other_runs_checkpoint_is_refused(tmp_path, field, value):
    p = str(tmp_path / "ck.json")
    save_checkpoint(p, KEY, 64, np.zeros(3, dtype=np.int64), 0.1)
    other = dict(KEY, **{field: value})
    with pytest.raises(SystemExit, match=field):
        load_checkpoint(p, other)


def test_version_and_range_are_checked(tmp_path):
    p = str(tmp_path / "ck.json")
    save_checkpoint(p, KEY, 64, np.zeros(3, dtype=np.int64), 0.1)
    d = json.load(open(p))
    d["version"] = CHECKPOINT_VERSION + 1
    json.dump(d, open(p, "w"))
    with pytest.raises(SystemExit, match="version"):
        load_checkpoint(p, KEY)
    d["version"] = CHECKPOINT_VERSION
    d["done"] = KEY["mine"] + 1
    json.dump(d, open(p, "w"))
    with pytest.raises(SystemExit, match="range"):
        load_checkpoint(p, KEY)


def test_flags_need_a_checkpoint_path():
    from dsce.simulate import main
    with pytest.raises(SystemExit, match="--checkpoint"):
        main(["--resume"])
    with pytest.raises(SystemExit, match="--checkpoint"):
        main(["--stop-after", "64"])
