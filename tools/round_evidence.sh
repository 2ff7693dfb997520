#!/bin/bash
# Round-end evidence on one box: the whole GPU suite, the default bench line, every config line,
# and a kernel trace + stats of the c4 d=3 sumcheck. Each step has its own time limit; the first
# failure ends the script. Output: gpurun_out/re_*
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/re_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/re_tests.log; exit 1; }
tail -1 gpurun_out/re_tests.log
timeout -k 10 400 python bench.py > gpurun_out/re_bench.json 2> gpurun_out/re_bench.err || { echo "bench failed"; tail -20 gpurun_out/re_bench.err; exit 1; }
cat gpurun_out/re_bench.json
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/re_configs.jsonl 2> gpurun_out/re_configs.err || { echo "configs failed"; tail -20 gpurun_out/re_configs.err; exit 1; }
cat gpurun_out/re_configs.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/re_sc_prof" -o run -- python3 "$R/tools/bench_configs.py" --only c4 --sc-d 3 > "$R/gpurun_out/re_sc_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/re_sc_prof.log"; exit 1; }
echo "round evidence done"
