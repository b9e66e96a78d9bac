"""CPU: the MEX gateway (channel-estimation_amd/matlab/dsce_mex.c) compiled
against a test-only mex.h stand-in and a recording stub of the C-ABI, run
under AddressSanitizer: every command checks its argument count and classes,
and every output is sized from dsce_scheme_dims (the stub writes exactly what
the engine writes, so an undersized output would be a reported heap overflow).
MATLAB itself is not in the image; this checks the gateway's own logic."""
import os
import re
import shutil
import subprocess

import pytest

import harness

MEX = os.path.join(harness.ROOT, "tests", "mex")
GATEWAY = os.path.join(harness.PKG, "matlab", "dsce_mex.c")


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    d = tmp_path_factory.mktemp("mex")
    exe = str(d / "drv")
    subprocess.run(["gcc", "-std=c11", "-g", "-O1", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-DMATLAB_MEX_FILE", "-D_GNU_SOURCE", "-I", MEX, "-I", os.path.join(harness.ROOT, "include"),
                    GATEWAY, os.path.join(MEX, "mex_stub.c"), os.path.join(MEX, "driver.c"), "-o", exe, "-lm"],
                   check=True)
    out = subprocess.run([exe], capture_output=True, text=True, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"),
                         timeout=120)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "AddressSanitizer" not in out.stderr, out.stderr[-3000:]
    res = {}
    for m in re.finditer(r"^(\w+) -> (OK|ERR) ?(\S*)$", out.stdout, re.M):
        res[m.group(1)] = (m.group(2), m.group(3))
    return res


def test_outputs_sized_from_engine_state(results):
    assert results["run"] == ("OK", "5x28")                               # [iter+1, snr, 2, 2, schemes]
    assert results["mmse_onetap_documented_5_args"] == ("OK", "336x1")   # INTEGRATION.md's PSACE call
    assert results["mmse_onetap_3_vectors_real"] == ("OK", "336x3")
    assert results["get_W"] == ("OK", "1806336x1")                       # LK^2 NP
    assert results["channel_realise"] == ("OK", "540x2")
    assert results["add_scheme"] == ("OK", "1x1")
    assert results["scheme_dims"] == ("OK", "1x9")
    for k in ("set_interpolation", "set_option", "set_channel", "create", "destroy"):
        assert results[k][0] == "OK", k


def test_arity_and_argument_checks(results):
    usage = ("run_old_7_args", "mmse_onetap_4_args", "mmse_onetap_old_6_args", "get_W_old_5_args",
             "channel_realise_old_5_args", "add_scheme_15_args", "scheme_dims_2_outputs", "unknown")
    for k in usage:
        assert results[k] == ("ERR", "dsce:usage"), (k, results[k])
    args = ("mmse_onetap_wrong_np", "get_W_scheme_0", "add_scheme_bad_Q", "add_scheme_bad_dataIdx",
            "set_interpolation_bad", "set_option_bad_name", "set_channel_fractional_N")
    for k in args:
        assert results[k] == ("ERR", "dsce:args"), (k, results[k])
    assert results["run_before_create"] == ("ERR", "dsce:state")
    assert results["after_destroy"] == ("ERR", "dsce:state")
