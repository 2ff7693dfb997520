#!/bin/bash
# Headline evidence for one build: the bench line (no CPU / config-5 legs unless HP_FULL=1) and a
# rocprofv3 kernel trace + stats of the same command, into gpurun_out/hp_*. Own time limit per step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
ARGS=${HP_ARGS:---no-cpu --no-c5 --no-configs --steps 20 --warmup 3}
timeout -k 10 300 python bench.py $ARGS > gpurun_out/hp_bench.json 2> gpurun_out/hp_bench.err || { echo "bench failed"; tail -20 gpurun_out/hp_bench.err; exit 1; }
cat gpurun_out/hp_bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/hp_prof" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/hp_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/hp_prof.log"; exit 1; }
echo "headline_prof done"
