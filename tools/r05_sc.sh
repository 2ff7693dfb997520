#!/bin/bash
# Round-5 sumcheck check: GPU sumcheck parity tests, then c4 (2^24, d = 2/3/4) for the libraries in
# AB_LIBS (tools/ab_libs.sh), each twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py tests/test_fixtures.py tests/test_distributed.py tests/test_gpu_rccl_world1.py -m gpu > gpurun_out/r05_sc_tests.txt 2>&1 || { tail -40 gpurun_out/r05_sc_tests.txt; exit 1; }
tail -2 gpurun_out/r05_sc_tests.txt
AB_CONFIGS=c4 tools/ab_libs.sh && AB_CONFIGS=c4 tools/ab_libs.sh
