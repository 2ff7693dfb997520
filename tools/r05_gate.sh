#!/bin/bash
# Pre-enqueued (gated) sumcheck folds: GPU sumcheck parity (incl. the gated edge cases), then c4 d=3
# alternated between this tree and $ALT (the library before the change)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_sumcheck.py tests/test_distributed.py tests/test_gpu_rccl_world1.py tests/test_fixtures.py -m gpu > gpurun_out/r05_gate_tests.txt 2>&1 || { tail -40 gpurun_out/r05_gate_tests.txt; exit 1; }
tail -1 gpurun_out/r05_gate_tests.txt
CMD="python3 tools/bench_configs.py --only c4 --sc-d 3 2>&1 | grep -o '\"ms\": [0-9.]*'" REPS=${REPS:-3} tools/ab.sh
