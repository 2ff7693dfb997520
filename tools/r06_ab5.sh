#!/bin/bash
# Round 6: the register-tile passes' LDS staging unpadded (32-word block slots, 16-byte chunks
# XOR-swizzled: 32 KB instead of 36.9 KB per work-group, BN_RR_SWZ -> lib-x1), and on top of it the
# first GF(2^8) pass forced to five waves per SIMD (BN_RR_OCC_FIRST=5 -> lib-x2), against the product
# library. The switches are tools/patches/r06_rr_staging.patch (measured slower, not in the source):
# git apply it, make -C binius-ntt_amd BUILD=build-x1 LIBDIR=lib-x1 EXTRA=-DBN_RR_SWZ (and x2 with
# EXTRA="-DBN_RR_SWZ -DBN_RR_OCC_FIRST=5"), git apply -R. Parity of both first (NTT + fixture tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for x in x1 x2; do
  BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-$x/libbinius_ntt_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_ntt.py tests/test_fixtures.py > gpurun_out/parity_$x.txt 2>&1 || { tail -20 gpurun_out/parity_$x.txt; exit 1; }
  echo "parity $x: $(tail -1 gpurun_out/parity_$x.txt)"
done
for rep in 1 2 3; do
  for x in lib x1 x2; do
    if [[ $x == lib ]]; then unset BINIUS_NTT_AMD_LIB; else export BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-$x/libbinius_ntt_amd.so; fi
    echo "== $x"
    BENCH_ARGS=--no-c5 timeout -k 10 120 tools/bench_brief.sh || exit 1
    timeout -k 10 120 python tools/bench_configs.py --only c3 2>/dev/null | grep '"c3"' | python3 -c "import sys,json; print('c3 ms %.4f' % json.loads(sys.stdin.read())['ms'])" || exit 1
  done
done
