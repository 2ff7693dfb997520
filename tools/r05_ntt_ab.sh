#!/bin/bash
# NTT parity (GF(2^128) tests + MD5 tables) of the in-tree library, then headline A/B against $ALT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ntt.py tests/test_fixtures.py -m gpu > gpurun_out/r05_ntt_tests.txt 2>&1 || { tail -30 gpurun_out/r05_ntt_tests.txt; exit 1; }
tail -1 gpurun_out/r05_ntt_tests.txt
CMD="BENCH_ARGS=--no-c5 tools/bench_brief.sh" REPS=${REPS:-3} tools/ab.sh 2>&1 | grep -v amdgpu.ids
