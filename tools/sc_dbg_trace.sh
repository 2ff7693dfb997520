#!/bin/bash
# Per-round c4 timelines with the development library (make BN_DEV=1) under BN_SC_DBG settings
# (SC_DBGS = space-separated values; bit 1 = no products: the kernels' memory-and-LDS floor).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export BINIUS_NTT_AMD_LIB="$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so"
for v in ${SC_DBGS:-0 2}; do
  echo "== BN_SC_DBG=$v"
  BN_SC_DBG=$v "$R/tools/sc_trace.sh" > /dev/null || exit 1
  cat "$R/gpurun_out/sc_rounds.txt"
done
