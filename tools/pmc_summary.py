#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc_*/run_counter_collection.csv) per kernel.

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of wide coalesced
streaming reads on gfx950 -> doubled here; WRITE_SIZE reads exact for 16-B stores. Both are
in KiB. Prints the per-kernel mean per dispatch and writes gpurun_out/pmc_summary.json.
With --traffic LOG_H it also writes profiles/pmc_traffic.json: {LOG_H: HBM bytes per launch of
the headline NTT's dominant kernel (the bottom pass, antt_bs_pass<4, 2, ...>)}, read by bench.py.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    traffic_log_h = None
    if "--traffic" in args:
        i = args.index("--traffic")
        traffic_log_h = args[i + 1]
        del args[i:i + 2]
    root = args[0] if args else os.path.join(ROOT, "gpurun_out")
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmc_*", "run_counter_collection.csv")):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            per[(row["Dispatch_Id"], row["Kernel_Name"])][row["Counter_Name"]] += float(row["Counter_Value"])
        for (_, k), cs in per.items():
            for c, v in cs.items():
                acc[k][c].append(v)
    out = {}
    for k, cs in acc.items():
        if "rocclr" in k:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in m:
            m["HBM_READ_BYTES_corrected"] = 2 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            m["HBM_WRITE_BYTES"] = m["WRITE_SIZE"] * 1024
        out[k] = m
        print(k)
        for c in sorted(m):
            print("   %-28s %.4g" % (c, m[c]))
    with open(os.path.join(root, "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    if traffic_log_h:
        dom = [k for k in out if "antt_bs_pass<4, 2" in k]
        if dom and "HBM_READ_BYTES_corrected" in out[dom[0]] and "HBM_WRITE_BYTES" in out[dom[0]]:
            m = out[dom[0]]
            path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            cur = json.load(open(path)) if os.path.exists(path) else {}
            cur[traffic_log_h] = m["HBM_READ_BYTES_corrected"] + m["HBM_WRITE_BYTES"]
            cur["_kernel_" + traffic_log_h] = dom[0]
            cur["_read_bytes_" + traffic_log_h] = m["HBM_READ_BYTES_corrected"]
            cur["_write_bytes_" + traffic_log_h] = m["HBM_WRITE_BYTES"]
            with open(path, "w") as f:
                json.dump(cur, f, indent=1)
            print("traffic per launch of %s: %.4g B" % (dom[0], cur[traffic_log_h]))


def headline(root, log_h, out_dir):
    """Per-pass counters of the headline transform (kernel variant 1: antt_bs_pass<4, ROLE, ...>;
    with three passes ROLE 0/1/2 = pass 0/1/2) -> out_dir/pmc_summary.json and pmc_traffic.json,
    keyed "log_h=N" -> pass index, as bench.py reads them."""
    with open(os.path.join(root, "pmc_summary.json")) as f:
        summ = json.load(f)
    per_pass, traffic = {}, {}
    for k, m in summ.items():
        if "antt_bs_pass<4, " not in k:
            continue
        role = int(k.split("antt_bs_pass<4, ")[1].split(",")[0])
        per_pass[str(role)] = dict(m, kernel=k)
        if "HBM_READ_BYTES_corrected" in m and "HBM_WRITE_BYTES" in m:
            traffic[str(role)] = m["HBM_READ_BYTES_corrected"] + m["HBM_WRITE_BYTES"]
    key = "log_h=%d" % log_h
    for name, data in (("pmc_summary.json", per_pass), ("pmc_traffic.json", traffic)):
        path = os.path.join(out_dir, name)
        cur = json.load(open(path)) if os.path.exists(path) else {}
        cur[key] = data
        with open(path, "w") as f:
            json.dump(cur, f, indent=1)
    print("headline %s: passes %s, traffic %s" % (key, sorted(per_pass), traffic))


def lib_sha256():
    import hashlib
    path = os.path.join(ROOT, "binius-ntt_amd", "lib", "libbinius_ntt_amd.so")
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def kernels(root, out_path, note):
    """Per-kernel counters keyed by the exact (demangled) kernel name, stamped with the SHA-256 of
    the library that was profiled: bench.py uses an entry only when its own library has the same
    hash and the pass it reports launched exactly that kernel (a kernel change makes it null)."""
    with open(os.path.join(root, "pmc_summary.json")) as f:
        summ = json.load(f)
    ks = {}
    for k, m in summ.items():
        e = dict(m)
        if "HBM_READ_BYTES_corrected" in m and "HBM_WRITE_BYTES" in m:
            e["HBM_BYTES"] = m["HBM_READ_BYTES_corrected"] + m["HBM_WRITE_BYTES"]
        ks[k] = e
    doc = {"lib_sha256": lib_sha256(), "note": note,
           "units": "per dispatch (mean over the profiled dispatches); FETCH_SIZE/WRITE_SIZE in KiB, "
                    "HBM_BYTES = 2 x FETCH_SIZE + WRITE_SIZE in bytes (gfx950 correction, MI355X_MICROARCH.md)",
           "kernels": ks}
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote %s (%d kernels, lib %s)" % (out_path, len(ks), doc["lib_sha256"][:16]))


if __name__ == "__main__":
    # --kernels OUT_PATH NOTE [ROOT]: per-kernel file keyed by exact name + library hash
    if "--kernels" in sys.argv:
        i = sys.argv.index("--kernels")
        out_path, note = sys.argv[i + 1], sys.argv[i + 2]
        rest = sys.argv[1:i] + sys.argv[i + 3:]
        sys.argv = [sys.argv[0]] + rest
        main()
        kernels(rest[0] if rest else os.path.join(ROOT, "gpurun_out"), out_path, note)
        sys.exit(0)
    # --headline LOG_H OUT_DIR [ROOT]: summarise ROOT's pmc_* runs, then write the per-pass files
    if "--headline" in sys.argv:
        i = sys.argv.index("--headline")
        log_h, out_dir = int(sys.argv[i + 1]), sys.argv[i + 2]
        rest = sys.argv[1:i] + sys.argv[i + 3:]
        sys.argv = [sys.argv[0]] + rest
        main()
        headline(rest[0] if rest else os.path.join(ROOT, "gpurun_out"), log_h, out_dir)
    else:
        main()
