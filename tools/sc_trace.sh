#!/bin/bash
# rocprofv3 kernel trace of the c4 sumcheck (2^24 evals, d=3) and its per-round timeline
# (kernel durations, idle gaps) -> gpurun_out/sc_trace/, gpurun_out/sc_rounds.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/sc_trace" -o run -- python3 "$R/tools/bench_configs.py" --only c4 --sc-d 3 > "$R/gpurun_out/sc_trace.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/sc_trace.log"; exit 1; }
grep '"c4"' "$R/gpurun_out/sc_trace.log" | head -3
python3 "$R/tools/sc_round_gaps.py" "$R/gpurun_out/sc_trace/run_kernel_trace.csv" 24 > "$R/gpurun_out/sc_rounds.txt" && cat "$R/gpurun_out/sc_rounds.txt"
