#!/bin/bash
# Round-4 first check on one box: the GPU suite, the default bench line, the reference sumcheck
# benchmark driver (Memcpy / Transpose / Raw phases). Each GPU step has its own time limit; the
# first failure ends the script. Output: gpurun_out/r04c_*
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -s > gpurun_out/r04c_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r04c_tests.log; exit 1; }
tail -1 gpurun_out/r04c_tests.log
grep EXCHANGE gpurun_out/r04c_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || { echo "bench failed"; tail -20 gpurun_out/r04c_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04c_bench.json'));print(d['ms_per_step'],d['roofline']['frac'],d['config']['output_check'],d['roofline']['pass_ms'])"
bash tools/run_benchmark_sumcheck.sh > /dev/null || { echo "benchmark_sumcheck failed"; tail -20 gpurun_out/benchmark_sumcheck.txt; exit 1; }
tail -2 gpurun_out/benchmark_sumcheck.txt
echo "r04 check done"
