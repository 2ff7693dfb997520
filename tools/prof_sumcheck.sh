#!/bin/bash
# rocprofv3 kernel trace of the sumcheck config (c4, d=3) -> gpurun_out/prof_sc/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_sc" -o run -- python3 "$R/tools/bench_configs.py" --only c4 --sc-d ${SC_D:-3} > "$R/gpurun_out/prof_sc.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_sc.log"; exit 1; }
cat "$R/gpurun_out/prof_sc/run_kernel_stats.csv"
