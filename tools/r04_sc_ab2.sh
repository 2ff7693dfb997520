#!/bin/bash
# Sumcheck candidate (the in-tree product library) on one box: the sumcheck GPU tests, then an A/B
# of c4 (AB_SCD, default d=3) against lib-x (two passes), then a kernel trace of the candidate.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/scab2_tests.log 2>&1 || { echo "sumcheck tests failed"; tail -40 gpurun_out/scab2_tests.log; exit 1; }
tail -1 gpurun_out/scab2_tests.log
for rep in 1 2; do
AB_LIBS="binius-ntt_amd/lib-x/libbinius_ntt_amd.so lib" AB_CONFIGS=c4 AB_SCD=${AB_SCD:-3} bash tools/ab_libs.sh || exit 1
done
bash tools/sc_trace.sh | tail -26
