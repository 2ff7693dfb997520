#!/bin/bash
# One GPU round trip: parity tests, short bench, rocprofv3 kernel trace. Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-pytest,bench,prof}
if [[ $STEPS == *pytest* ]]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-420} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-configs --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  find "$R/gpurun_out/prof" -name "*stats*" | head
fi
echo "gpu_check done"
