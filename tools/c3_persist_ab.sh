#!/bin/bash
# C3 (one 2^20 GF(2^128) transform): the default three launches (variant 5), variant 1's three
# launches, and variant 1's passes as ONE persistent launch with grid barriers (BN_PERSIST3, dev
# build), alternated; parity of the persistent launch checked against the oracle first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
BN_PERSIST3=1 BN_ANTT_VARIANT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py -m gpu -k "gf128 and not 26" > gpurun_out/c3_persist_tests.txt 2>&1 || { tail -20 gpurun_out/c3_persist_tests.txt; exit 1; }
tail -1 gpurun_out/c3_persist_tests.txt
line() { timeout -k 10 120 python tools/bench_configs.py --only c3 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'): d=json.loads(l); print('%.4f ms' % d['ms'])"; }
for rep in 1 2 3; do
  echo "default (variant 5): $(line)"
  echo "variant 1, 3 launches: $(BN_ANTT_VARIANT=1 line)"
  echo "variant 1, persistent: $(BN_ANTT_VARIANT=1 BN_PERSIST3=1 line)"
done
