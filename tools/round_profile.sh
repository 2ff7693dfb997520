#!/bin/bash
# Round evidence for profiles/rNN (default r06) on one box, for the library as built in this tree:
#   1. PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the headline bench and of the config-2 loops, each
#      counter group in its own rocprofv3 run (MI355X_MICROARCH.md), summarised per kernel name and
#      stamped with the library's SHA-256 -> profiles/$R/pmc_kernels.json (read by bench.py)
#   2. rocprofv3 --kernel-trace --stats of the default headline bench -> profiles/$R/headline_*
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
RN=${ROUND_DIR:-r06}
cd "$R"
mkdir -p gpurun_out "profiles/$RN"
PMC_GROUPS=fetch,write,sq,stall PMC_TAG=hl_ PMC_ARGS="--no-cpu --no-configs --no-c5 --steps 3 --warmup 1" bash tools/pmc.sh || exit 1
PMC_GROUPS=sq PMC_TAG=c2_ PMC_SCRIPT=tools/bench_configs.py PMC_ARGS="--only c2" bash tools/pmc.sh || exit 1
python3 tools/pmc_summary.py --kernels "profiles/$RN/pmc_kernels.json" "headline bench (default variant) + config-2 loops" gpurun_out > gpurun_out/pmc_summary.txt || exit 1
# only gpurun_out/ comes back from the box: keep a copy there (copy it into profiles/$RN by hand)
mkdir -p "gpurun_out/profile_$RN" && cp "profiles/$RN/pmc_kernels.json" "gpurun_out/profile_$RN/"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/rp_prof" -o run -- python3 "$R/bench.py" --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 > "$R/gpurun_out/rp_bench.json" 2> "$R/gpurun_out/rp_prof.log" || { echo "rocprof failed"; tail -20 "$R/gpurun_out/rp_prof.log"; exit 1; }
cd "$R"
P="gpurun_out/profile_$RN"
cp gpurun_out/rp_prof/run_kernel_stats.csv "$P/headline_kernel_stats.csv"
cp gpurun_out/rp_prof/run_kernel_trace.csv "$P/headline_kernel_trace.csv"
cp gpurun_out/rp_bench.json "$P/headline_bench_under_rocprof.json"
python3 tools/trace_passes.py "$P/headline_kernel_trace.csv" > "$P/headline_trace_passes.json" 2>/dev/null || true
echo "round_profile done"
