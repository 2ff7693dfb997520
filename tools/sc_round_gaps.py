"""Per-round timeline of the last sumcheck protocol run in a rocprofv3 kernel trace
(tools/sc_trace.sh): kernel durations and the idle gaps between them, in microseconds.
  python tools/sc_round_gaps.py <run_kernel_trace.csv> <nvars>"""
import csv
import re
import sys


def main():
    path, nvars = sys.argv[1], int(sys.argv[2])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "sc_" not in name:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    # a protocol run starts with round 0's messages launch, the only messages launch not preceded
    # by a fold (the last rounds may run inside one sc_server launch): take the last such start
    starts = [i for i, r in enumerate(rows)
              if "sc_messages" in r[2] and (i == 0 or "sc_fold" not in rows[i - 1][2])]
    first = starts[-1]
    run = rows[first:]
    t0 = run[0][0]
    busy = sum(e - s for s, e, _ in run)
    wall = run[-1][1] - t0
    print("kernels %d  wall %.1f us  busy %.1f us  idle %.1f us" % (len(run), wall / 1e3, busy / 1e3, (wall - busy) / 1e3))
    prev_end = None
    rnd = 0
    line = []
    for s, e, name in run:
        m = re.search(r"sc_\w+(<[^>]*>)?", name)
        short = m.group(0) if m else name[:24]
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        line.append("%s %.1f (+%.1f)" % (short, (e - s) / 1e3, gap))
        prev_end = e
        if "sc_fold" in name or "sc_server" in name:
            print("round %2d: %s" % (rnd, "  ".join(line)))
            line = []
            rnd += 1
    if line:
        print("round %2d: %s" % (rnd, "  ".join(line)))


if __name__ == "__main__":
    main()
