#!/bin/bash
# Round-5 GPU check: the sharded-exchange tests (RCCL world 1, gloo world 2), GF(2^128) NTT parity
# of an experiment library ($EXP_LIB) and an A/B of the headline against it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -s tests/test_gpu_rccl_world1.py tests/test_distributed.py -m gpu > gpurun_out/r05_dist_tests.txt 2>&1 || { tail -30 gpurun_out/r05_dist_tests.txt; exit 1; }
grep -E "EXCHANGE|passed|failed" gpurun_out/r05_dist_tests.txt
if [ -n "$EXP_LIB" ]; then
  BINIUS_NTT_AMD_LIB=$PWD/$EXP_LIB timeout -k 10 600 $T tests/test_gpu_ntt.py -m gpu -k "gf128 or md5 or fixtures" > gpurun_out/r05_exp_ntt.txt 2>&1 || { tail -30 gpurun_out/r05_exp_ntt.txt; exit 1; }
  tail -2 gpurun_out/r05_exp_ntt.txt
  CMD="BENCH_ARGS=--no-c5 tools/bench_brief.sh" ALT="$EXP_LIB" REPS=${REPS:-3} tools/ab.sh 2>&1 | grep -v amdgpu.ids
fi
