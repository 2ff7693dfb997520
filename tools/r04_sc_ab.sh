#!/bin/bash
# Sumcheck changes on one box: the sumcheck GPU tests on the candidate library (lib-x), an A/B of
# c4 d=3 over lib-base / lib / lib-x (two passes), then the host-side round timing.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-x/libbinius_ntt_amd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_sumcheck.py tests/test_gpu_rccl_world1.py -m gpu -x -q -s --timeout 240 --timeout-method thread > gpurun_out/scab_tests.log 2>&1 || { echo "sumcheck tests failed"; tail -40 gpurun_out/scab_tests.log; exit 1; }
tail -1 gpurun_out/scab_tests.log
grep EXCHANGE gpurun_out/scab_tests.log
for rep in 1 2; do
AB_LIBS="binius-ntt_amd/lib-base/libbinius_ntt_amd.so lib binius-ntt_amd/lib-x/libbinius_ntt_amd.so" AB_CONFIGS=c4 AB_SCD=${SC_D:-3} bash tools/ab_libs.sh || exit 1
done
timeout -k 10 200 python tools/sc_host_timing.py > gpurun_out/sc_host.txt 2>&1 || { echo "host timing failed"; tail -5 gpurun_out/sc_host.txt; exit 1; }
cat gpurun_out/sc_host.txt
