"""CPU: the bench line's derived fields (bench.py) — the limiter from a stamped
PMC summary, the dominant-by-time entry, the committed evidence files' shape —
without a GPU.  The numbers the GPU produces are checked on the box
(`-m gpu`); here only the arithmetic that turns counters into the line."""
import glob
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pmc(valu, mfma_cycles, grbm=8e6, wave_cycles=4e9, wait=1e9, hbm=None, dur_ns=2.5e6):
    return {"sq_per_launch": {"GRBM_GUI_ACTIVE": grbm, "SQ_INSTS_VALU": valu, "SQ_VALU_MFMA_BUSY_CYCLES": mfma_cycles,
                              "SQ_WAVE_CYCLES": wave_cycles, "SQ_WAIT_INST_ANY": wait, "SQ_INSTS_MFMA": 1e6},
            "hbm_bytes_per_launch": hbm, "avg_duration_ns_rocprof": dur_ns}


def test_limiter_is_the_shared_fp64_issue_when_neither_pipe_alone_fills_it():
    cyc = 8e6 / 8.0
    # VALU 0.5 and MFMA 0.4 of the SIMDs' cycles: together 0.9 -> FP64 issue
    pmc = _pmc(valu=0.5 * bench.SIMDS * cyc / 4.0, mfma_cycles=0.4 * bench.SIMDS * cyc)
    d = bench.derive_limiter(pmc, 30.0, 2.5)
    assert abs(d["valu_issue"] - 0.5) < 1e-12 and abs(d["mfma_busy"] - 0.4) < 1e-12
    assert d["limiter"].startswith("FP64 issue") and abs(d["issue"] - 0.9) < 1e-12
    # VALU alone at 0.92 -> VALU issue
    d = bench.derive_limiter(_pmc(valu=0.92 * bench.SIMDS * cyc / 4.0, mfma_cycles=0.0), None, 2.5)
    assert d["limiter"] == "VALU issue"
    # HBM: 20 GB in 2.5 ms = 8 TB/s
    d = bench.derive_limiter(_pmc(valu=0.1 * bench.SIMDS * cyc / 4.0, mfma_cycles=0.0, hbm=20e9), None, 2.5)
    assert d["limiter"] == "HBM bandwidth" and abs(d["hbm"] - 20e9 / 2.5e-3 / (bench.HBM_PEAK_GBS * 1e9)) < 1e-12
    # no counters -> no limiter
    assert bench.derive_limiter(None, 1.0, 1.0) is None
    assert bench.derive_limiter({"sq_per_launch": {}}, 1.0, 1.0) is None


def test_dominant_by_time_names_another_group_only():
    kernels = {"k_mic_data": {"ms_per_step": 2.5, "share": 0.3, "tflops": 27.0, "frac_fp64": 0.34},
               "perfect_ic": {"ms_per_step": 2.6, "share": 0.31, "tflops": 25.0, "frac_fp64": 0.32,
                              "limiter": "FP64 issue"}}
    d = bench.dominant_by_time(kernels, "k_mic_data")
    assert d["kernel"] == "perfect_ic" and d["ms_per_step"] == 2.6 and d["limiter"] == "FP64 issue"
    assert bench.dominant_by_time(kernels, "perfect_ic") is None
    assert bench.dominant_by_time({}, "k_mic_data") is None


def test_source_hash_covers_the_engine_sources():
    h = bench.source_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    assert h == bench.source_hash()


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "profiles", "r04h*_bench.json"))))
def test_committed_bench_lines_keep_the_contract(path):
    """Every committed final-round bench line: the driver's keys, a roofline
    fraction in (0, 1], the CPU baseline object, and a stamped PMC source."""
    d = json.load(open(path))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, (path, k)
    r = d["roofline"]
    assert 0.0 < r["frac"] <= 1.0 and r["unit"] == "TFLOP/s"
    assert r["bound"] in ("mfma", "hbm", "fp64 (VALU+MFMA shared)")
    assert r["traffic"] and r["traffic_source"].startswith("profiles/") and len(r["source_hash"]) == 16
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1
    assert d["dtype"] == "f64" and d["n_gpus"] == 1
