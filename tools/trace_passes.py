#!/usr/bin/env python3
"""Per-pass mean durations of the headline NTT's launches from a rocprofv3 kernel trace of
`bench.py --no-cpu --no-c5 --no-configs --steps K --warmup W` (tools/headline_prof.sh).

bench.py launches every pass kernel in this order: W warm-up transforms, max(5, min(K, 20))
transforms with events between the passes (pass_ms_inloop), then each pass 1 + max(10, min(K, 40))
times back to back (bn_antt_time_passes, pass_ms), then the K timed transforms, then apply_e2e.
This prints the mean duration of each phase's launches per pass kernel, so the bench's
`roofline.pass_ms` / `kernel_ms` can be checked against the profiler's clock.

  python tools/trace_passes.py gpurun_out/hp_prof/run_kernel_trace.csv [K] [W]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    w = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ev = max(5, min(k, 20))
    iso = 1 + max(10, min(k, 40))
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    for r in rows:
        if any(t in r["Kernel_Name"] for t in ("antt_bs_pass", "antt_rt_pass", "antt_rr_pass")):
            per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for name, d in sorted(per.items(), key=lambda kv: kv[0]):
        phases = {"warmup": d[:w], "inloop_events": d[w:w + ev], "isolated": d[w + ev + 1:w + ev + iso],
                  "timed": d[w + ev + iso:w + ev + iso + k]}
        out[name] = {p: (sum(v) / len(v) if v else None) for p, v in phases.items()}
        out[name]["launches"] = len(d)
    tot = sum(v["timed"] for v in out.values() if v["timed"])
    out["sum_timed_ms"] = tot
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
