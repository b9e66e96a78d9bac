"""CPU: the MEX gateway (channel-estimation_amd/matlab/dsce_mex.c) compiled
against a test-only mex.h stand-in and a recording stub of the C-ABI, run
under AddressSanitizer: every command checks its argument count and classes,
and every output is sized from dsce_scheme_dims (the stub writes exactly what
the engine writes, so an undersized output would be a reported heap overflow).
The gateway is built twice: for MATLAB's interleaved complex API (R2018a+) and
for the split real / imaginary planes of R2013b / R2016a (README.md:19-20).
Every dsce_mex(...) call in INTEGRATION.md and in the PSACE 'MMSE' patch is
replayed through it, so the documented binding cannot drift from the gateway.
MATLAB itself is not in the image; this checks the gateway's own logic."""
import os
import re
import shutil
import subprocess

import pytest

import harness

MEX = os.path.join(harness.ROOT, "tests", "mex")
GATEWAY = os.path.join(harness.PKG, "matlab", "dsce_mex.c")


INTEGRATION = os.path.join(harness.ROOT, "INTEGRATION.md")
PATCH = os.path.join(harness.PKG, "matlab", "psace_mmse.patch")


def _build(d, split):
    exe = str(d / ("drv_split" if split else "drv"))
    subprocess.run(["gcc", "-std=c11", "-g", "-O1", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-Werror=implicit-function-declaration", "-DMATLAB_MEX_FILE", "-D_GNU_SOURCE"]
                   + (["-DDSCE_TEST_SPLIT"] if split else [])
                   + ["-I", MEX, "-I", os.path.join(harness.ROOT, "include"),
                      GATEWAY, os.path.join(MEX, "mex_stub.c"), os.path.join(MEX, "driver.c"), "-o", exe, "-lm"],
                   check=True)
    return exe


def _run(exe, args=()):
    out = subprocess.run([exe, *args], capture_output=True, text=True,
                         env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"), timeout=120)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "AddressSanitizer" not in out.stderr, out.stderr[-3000:]
    res = {}
    for m in re.finditer(r"^(\S+) -> (OK|ERR) ?(\S*)$", out.stdout, re.M):
        res[m.group(1)] = (m.group(2), m.group(3))
    return res, out.stdout


@pytest.fixture(scope="module", params=["interleaved", "split"])
def built(request, tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    return _build(tmp_path_factory.mktemp("mex"), request.param == "split")


@pytest.fixture(scope="module")
def results(built):
    res, stdout = _run(built)
    assert "BAD" not in stdout, [l for l in stdout.splitlines() if "BAD" in l]
    assert stdout.count("check ") >= 6
    return res


# ---------------------------------------------------------------------------
# dsce_mex(...) calls of a MATLAB text: (command, number of inputs, outputs)
# ---------------------------------------------------------------------------
def _strip_comment(line):
    q = False
    for i, ch in enumerate(line):
        if ch == "'":
            q = not q
        elif ch == "%" and not q:
            return line[:i]
    return line


def _statements(text):
    out, cur = [], ""
    for line in text.splitlines():
        line = _strip_comment(line).rstrip()
        if line.endswith("..."):
            cur += line[:-3] + " "
            continue
        out.append(cur + line)
        cur = ""
    if cur:
        out.append(cur)
    return out


def _calls(text):
    calls = []
    for st in _statements(text):
        for m in re.finditer(r"dsce_mex\(", st):
            i, depth, q, args, a0 = m.end(), 1, False, [], m.end()
            while i < len(st) and depth:
                ch = st[i]
                if ch == "'":
                    q = not q
                elif not q and ch in "([{":
                    depth += 1
                elif not q and ch in ")]}":
                    depth -= 1
                    if depth == 0:
                        args.append(st[a0:i].strip())
                elif not q and ch == "," and depth == 1:
                    args.append(st[a0:i].strip())
                    a0 = i + 1
                i += 1
            assert depth == 0, "unbalanced dsce_mex call: " + st
            lhs = st[:m.start()].rstrip()
            nlhs = 0
            if lhs.endswith("=") and not lhs.endswith("=="):
                head = lhs[:-1].strip()
                nlhs = len(head.strip("[]").split(",")) if head.startswith("[") else 1
            calls.append((args[0].strip("'"), len(args), nlhs))
    return calls


def _integration_calls():
    text = open(INTEGRATION).read()
    code = "\n".join(re.findall(r"```matlab\n(.*?)```", text, re.S))
    inline = [c for c in re.findall(r"`(dsce_mex\([^`]*\))`", text) if "..." not in c]
    return _calls(code + "\n" + "\n".join(inline))


FF_PATCH = os.path.join(harness.PKG, "matlab", "fastfading_dsce.patch")
MOD_PATCH = os.path.join(harness.PKG, "matlab", "modulation_dsce.patch")


def _patch_calls(path=PATCH):
    plus = [l[1:] for l in open(path).read().splitlines() if l.startswith("+") and not l.startswith("+++")]
    return _calls("\n".join(plus))


def test_integration_md_calls_run_through_the_gateway(built):
    """Every dsce_mex(...) call INTEGRATION.md documents (and the one inside the
    PSACE 'MMSE' patch) is accepted by the gateway with that many inputs and
    outputs: a documented call the gateway rejects (round-2: 'run' with 7
    arguments) fails here."""
    calls = _integration_calls() + _patch_calls() + _patch_calls(FF_PATCH) + _patch_calls(MOD_PATCH)
    cmds = {c[0] for c in calls}
    assert {"create", "set_channel", "set_snr", "add_scheme", "build_mmse", "run", "bits_per_rep",
            "mmse_onetap", "set_interpolation", "set_noise_slot", "tx_matrices", "enable_mse", "get_mse",
            "channel_realise"} <= cmds, cmds
    assert ("run", 4, 1) in calls and ("mmse_onetap", 5, 1) in _patch_calls()
    assert {("set_channel", 7, 0), ("channel_realise", 3, 1)} <= set(_patch_calls(FF_PATCH))
    assert set(_patch_calls(MOD_PATCH)) == {("tx_matrices", 2, 2)}
    # create first (the gateway refuses any other command before it)
    triples = ["create:1:0"] + ["%s:%d:%d" % c for c in calls if c[0] != "create"]
    res, stdout = _run(built, ["replay", *triples])
    assert "BAD" not in stdout
    for t in triples:
        assert res.get(t, ("missing",))[0] == "OK", (t, res.get(t), stdout[-2000:])


def test_psace_patch_applies_to_the_reference(tmp_path):
    """The patch applies cleanly to the reference's class (when the reference
    is present: this container, not the GPU box) and leaves no error() stub."""
    ref = "/root/reference/+ChannelEstimation/PilotSymbolAidedChannelEstimation.m"
    if not os.path.exists(ref) or not shutil.which("patch"):
        pytest.skip("reference or patch(1) not available")
    d = tmp_path / "+ChannelEstimation"
    d.mkdir()
    shutil.copy(ref, d / "PilotSymbolAidedChannelEstimation.m")
    out = subprocess.run(["patch", "-p1", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    body = (d / "PilotSymbolAidedChannelEstimation.m").read_text()
    assert "Needs to be" not in body and body.count("dsce_mex('mmse_onetap'") == 1
    assert "numel(varargin) < 4" in body                  # the missing [SchemeId SNRIndex] is an error()


def test_fastfading_patch_applies_to_the_reference(tmp_path):
    """The FastFading shim (NewRealization routed to dsce_channel_realise,
    FastFading.m:194-250) applies cleanly to the reference's class and adds
    exactly one UseEngine method and one engine branch in NewRealization."""
    ref = "/root/reference/+Channel/FastFading.m"
    if not os.path.exists(ref) or not shutil.which("patch"):
        pytest.skip("reference or patch(1) not available")
    d = tmp_path / "+Channel"
    d.mkdir()
    shutil.copy(ref, d / "FastFading.m")
    out = subprocess.run(["patch", "-p1", "-i", FF_PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    body = (d / "FastFading.m").read_text(encoding="latin-1")
    assert body.count("function UseEngine( obj, Seed, FirstRealization )") == 1
    assert body.count("dsce_mex('channel_realise'") == 1 and body.count("dsce_mex('set_channel'") == 1


def test_outputs_sized_from_engine_state(results):
    assert results["run"] == ("OK", "5x28")                               # [iter+1, snr, 2, 2, schemes]
    assert results["mmse_onetap_documented_5_args"] == ("OK", "336x1")   # INTEGRATION.md's PSACE call
    assert results["mmse_onetap_3_vectors_real"] == ("OK", "336x3")
    assert results["get_W"] == ("OK", "1806336x1")                       # LK^2 NP
    assert results["channel_realise"] == ("OK", "540x2")
    assert results["add_scheme"] == ("OK", "1x1")
    assert results["scheme_dims"] == ("OK", "1x9")
    for k in ("set_interpolation", "set_option", "set_channel", "create", "destroy", "enable_mse"):
        assert results[k][0] == "OK", k
    # the object's properties reach dsce_tx_desc (mex_stub.c checks every field)
    assert results["tx_matrices_ofdm"] == ("OK", "540x336") and results["tx_matrices_fbmc"] == ("OK", "540x720")
    assert results["get_mse"] == ("OK", "5x7")                          # [iter+1, snr, scheme]
    assert results["structured_check"] == ("OK", "1x7")
    # a device vector makes one multi-device context (ABI 7); 'group_info' reports it
    assert results["group_info_single"] == ("OK", "1x1")
    assert results["create_multi_8"] == ("OK", "") and results["group_info_multi"] == ("OK", "1x8")
    assert results["run_multi"] == ("OK", "5x28") and results["create_again"][0] == "OK"


def test_arity_and_argument_checks(results):
    usage = ("run_old_7_args", "mmse_onetap_4_args", "mmse_onetap_old_6_args", "get_W_old_5_args",
             "channel_realise_old_5_args", "add_scheme_15_args", "scheme_dims_2_outputs", "unknown",
             "tx_matrices_3_outputs", "get_mse_extra_arg")
    for k in usage:
        assert results[k] == ("ERR", "dsce:usage"), (k, results[k])
    args = ("mmse_onetap_wrong_np", "get_W_scheme_0", "add_scheme_bad_Q", "add_scheme_bad_dataIdx",
            "set_interpolation_bad", "set_option_bad_name", "set_channel_fractional_N", "tx_matrices_not_object",
            "tx_matrices_real_signal", "tx_matrices_phydyas")
    for k in args:
        assert results[k] == ("ERR", "dsce:args"), (k, results[k])
    assert results["create_empty_devices"] == ("ERR", "dsce:args")
    assert results["run_before_create"] == ("ERR", "dsce:state")
    assert results["after_destroy"] == ("ERR", "dsce:state")


def test_modulation_patch_applies_to_the_reference(tmp_path):
    """The +Modulation shim (GetTXMatrix / GetRXMatrix of OFDM.m:184-218 and
    FBMC.m:318-354 routed to dsce_mex('tx_matrices')) applies
    cleanly to both reference classes: one UseEngine method and one engine
    branch in each of GetTXMatrix / GetRXMatrix per class."""
    ref = "/root/reference/+Modulation"
    if not os.path.exists(ref) or not shutil.which("patch"):
        pytest.skip("reference or patch(1) not available")
    d = tmp_path / "+Modulation"
    d.mkdir()
    for f in ("OFDM.m", "FBMC.m"):
        shutil.copy(os.path.join(ref, f), d / f)
    out = subprocess.run(["patch", "-p1", "-i", MOD_PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    for f in ("OFDM.m", "FBMC.m"):
        body = (d / f).read_text(encoding="latin-1")
        assert body.count("function UseEngine(obj, On)") == 1, f
        assert body.count("] = dsce_mex('tx_matrices', obj);") == 2, f
        assert body.count("~obj.PHY.TransmitRealSignal") == 2, f
