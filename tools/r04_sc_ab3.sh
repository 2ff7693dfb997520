#!/bin/bash
# Candidate sumcheck library in lib-x vs the in-tree product: sumcheck GPU tests on lib-x, then
# c4 d=2,3,4 A/B (two passes).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-x/libbinius_ntt_amd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/scab3_tests.log 2>&1 || { echo "sumcheck tests failed"; tail -40 gpurun_out/scab3_tests.log; exit 1; }
tail -1 gpurun_out/scab3_tests.log
for rep in 1 2; do
AB_LIBS="lib binius-ntt_amd/lib-x/libbinius_ntt_amd.so" AB_CONFIGS=c4 AB_SCD=${AB_SCD:-2,3,4} bash tools/ab_libs.sh 2>&1 | grep -v "compact input" || exit 1
done
