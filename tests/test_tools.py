"""Host-side checks of the measurement tools (no GPU): tools/trace_passes.py splits a rocprofv3
kernel trace of bench.py into its launch phases (warm-up, in-loop events, isolated pass loops,
timed transforms) exactly as bench.py orders them."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trace_passes_phases(tmp_path):
    k, w = 5, 2
    ev, iso = max(5, min(k, 20)), 1 + max(10, min(k, 40))
    names = ["void bn::antt_bs_pass<4, %d, 32, false>(bn::BsParams)" % r for r in range(3)]
    rows, t = [], 0

    def launch(r, dur):
        nonlocal t
        rows.append({"Kernel_Name": names[r], "Start_Timestamp": t, "End_Timestamp": t + dur})
        t += dur + 10

    phase_dur = {"warmup": 900, "inloop": 700, "isolated": 500, "timed": 400}
    for _ in range(w):
        for r in range(3):
            launch(r, phase_dur["warmup"] * (r + 1))
    for _ in range(ev):
        for r in range(3):
            launch(r, phase_dur["inloop"] * (r + 1))
    for r in range(3):
        for _ in range(iso):
            launch(r, phase_dur["isolated"] * (r + 1))
    for _ in range(k):
        for r in range(3):
            launch(r, phase_dur["timed"] * (r + 1))
    p = tmp_path / "trace.csv"
    with open(p, "w", newline="") as f:
        wr = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        wr.writeheader()
        wr.writerows(rows)
    out = json.loads(subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "trace_passes.py"),
                                              str(p), str(k), str(w)]))
    for r, n in enumerate(names):
        assert out[n]["warmup"] * 1e6 == phase_dur["warmup"] * (r + 1)
        assert out[n]["inloop_events"] * 1e6 == phase_dur["inloop"] * (r + 1)
        assert abs(out[n]["isolated"] * 1e6 - phase_dur["isolated"] * (r + 1)) < 1e-6
        assert abs(out[n]["timed"] * 1e6 - phase_dur["timed"] * (r + 1)) < 1e-6
    assert abs(out["sum_timed_ms"] * 1e6 - 400 * 6) < 1e-6
