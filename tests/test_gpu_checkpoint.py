"""GPU: checkpoint / resume of `python -m dsce.simulate`.
A run stopped after its first batch (--stop-after) and resumed from its
checkpoint counts exactly like the uninterrupted run — the Philox streams are
keyed by the global realisation index — and its MSE sums agree to rounding; a
resume under another seed is refused."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import harness

pytestmark = pytest.mark.gpu

ARGS = ["--config", "default", "--schemes", "ofdm", "--reps", "300", "--batch", "128", "--mse"]


def _sim(extra, check=True):
    env = dict(os.environ, PYTHONPATH=harness.PKG)
    return subprocess.run([sys.executable, "-m", "dsce.simulate", *ARGS, *extra], cwd=harness.PKG, env=env,
                          check=check, timeout=240, capture_output=True, text=True)


def test_resumed_run_counts_like_the_uninterrupted_run(tmp_path):
    whole, resumed, ck = tmp_path / "whole.json", tmp_path / "resumed.json", str(tmp_path / "ck.json")
    _sim(["--out", str(whole)])
    r = _sim(["--checkpoint", ck, "--stop-after", "128", "--out", str(resumed)])
    assert "stopped at realisation 128 of 300" in r.stdout and not resumed.exists()
    assert json.load(open(ck))["done"] == 128
    bad = _sim(["--checkpoint", ck, "--resume", "--seed", "1"], check=False)
    assert bad.returncode != 0 and "belongs to another run" in bad.stderr
    r = _sim(["--checkpoint", ck, "--resume", "--out", str(resumed)])
    assert "resumed from" in r.stdout
    a, b = json.load(open(whole)), json.load(open(resumed))
    np.testing.assert_array_equal(np.array(b["counts"]), np.array(a["counts"]))
    assert b["resumed"] is True and "resumed" not in a
    for s in a["nmse"]:
        np.testing.assert_allclose(np.array(b["nmse"][s]), np.array(a["nmse"][s]), rtol=1e-12)
