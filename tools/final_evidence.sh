#!/bin/bash
# Round-end evidence on one box: full GPU parity suite, PMC + rocprofv3 summaries for the library
# as built (tools/round_profile.sh), then the default bench line. Each GPU step is time-limited and
# the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
export ROUND_DIR=${ROUND_DIR:-r06}
bash tools/round_profile.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
cp gpurun_out/bench_default.json gpurun_out/profile_$ROUND_DIR/bench_default.json
cp gpurun_out/pytest_gpu.log gpurun_out/profile_$ROUND_DIR/gpu_tests.txt
echo "final_evidence done"
