#!/bin/bash
# Round 6: 6 + 6 + 12 (BN_FIRST_K=6: the register-tile GF(2^8) pass gives its lowest stage to the
# LDS-tile middle pass) against the default 7 + 5 + 12, development build, three alternating pairs;
# parity of the 6 + 6 + 12 plan first (the NTT tests that run the default variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
BN_FIRST_K=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ntt.py \
  -k "not register_tile and not variant and not lane_split" > gpurun_out/parity_6_6_12.txt 2>&1 || { tail -20 gpurun_out/parity_6_6_12.txt; exit 1; }
tail -1 gpurun_out/parity_6_6_12.txt
for rep in 1 2 3; do
  for k in 7 6; do
    echo "== first pass $k stages"
    BN_FIRST_K=$k BENCH_ARGS=--no-c5 timeout -k 10 120 tools/bench_brief.sh || exit 1
  done
done
