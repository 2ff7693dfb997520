#!/bin/bash
# Pass times of the development build with parts of the work skipped (BN_DEBUG_FLAGS: 1 no loads,
# 2 no stores, 3 neither): how much of each LDS-tile pass its HBM traffic costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
for rep in 1 2; do
  for f in 0 1 2 3; do
    echo "== flags $f"
    BN_DEBUG_FLAGS=$f BENCH_ARGS=--no-c5 timeout -k 10 120 tools/bench_brief.sh || exit 1
  done
done
