#!/bin/bash
# C3 (one 2^20 transform): the bottom pass on register tiles (default since round 5) vs LDS tiles
# (BN_RR_LAST=0, development build), parity first, then alternated timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py -m gpu -k "gf128" > gpurun_out/r05_rrlast_tests.txt 2>&1 || { tail -20 gpurun_out/r05_rrlast_tests.txt; exit 1; }
tail -1 gpurun_out/r05_rrlast_tests.txt
line() { timeout -k 10 120 python3 tools/bench_configs.py --only c3 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'): d=json.loads(l); print('%.4f ms' % d['ms'])"; }
for rep in 1 2 3; do
  echo "LDS-tile bottom: $(BN_RR_LAST=0 line)"
  echo "register-tile bottom (default): $(line)"
done
