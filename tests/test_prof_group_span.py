"""CPU: tools/prof_summary.group_span over synthetic rocprofv3 kernel traces —
the IC group's span per step is first start -> last end of the (k_pic_fft,
k_mic_pilot, k_mic_data) triple."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _trace(path, rows):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for name, t0, t1 in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": t0, "End_Timestamp": t1})


def test_group_span_triple(tmp_path):
    import prof_summary
    tri = tmp_path / "tri"
    _trace(str(tri), [("void dsce::k_jakes_grp<28, 16>(x)", 0, 50),
                      ("void dsce::k_pic_fft<2, 2, false, true, true>(x)", 100, 300),
                      ("void dsce::k_mic_pilot<2, 2, 16, false, true, true>(x)", 300, 420),
                      ("void dsce::k_mic_data<2, 2, 16, false, true, true>(x)", 420, 620),
                      ("void dsce::k_pic_fft<2, 2, false, true, true>(x)", 1000, 1210),
                      ("void dsce::k_mic_pilot<2, 2, 16, false, true, true>(x)", 1210, 1330),
                      ("void dsce::k_mic_data<2, 2, 16, false, true, true>(x)", 1330, 1540)])
    assert prof_summary.group_span(str(tri)) == (520 + 540) / 2
    assert prof_summary.group_span(str(tmp_path / "none")) is None
