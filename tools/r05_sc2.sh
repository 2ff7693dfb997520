#!/bin/bash
# sumcheck parity tests, the round server's per-round timing (dev build), c4 A/B over AB_LIBS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py tests/test_fixtures.py tests/test_distributed.py -m gpu > gpurun_out/r05_sc_tests.txt 2>&1 || { tail -40 gpurun_out/r05_sc_tests.txt; exit 1; }
tail -1 gpurun_out/r05_sc_tests.txt
BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so BN_SC_TIMING=1 timeout -k 10 300 python tools/bench_configs.py --only c4 --sc-d 3 > gpurun_out/r05_srv_timing.txt 2>&1 || exit 1
grep "server round" gpurun_out/r05_srv_timing.txt | tail -12
for rep in 1 2; do
for L in $AB_LIBS; do
  if [[ $L == lib ]]; then unset BINIUS_NTT_AMD_LIB; else export BINIUS_NTT_AMD_LIB=$PWD/$L; fi
  echo "== $L $(timeout -k 10 200 python tools/bench_configs.py --only c4 --sc-d 2,3,4 2>/dev/null | python3 -c "import sys,json
out=[]
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l)
        if 'ms' in d: out.append('%.3f'%d['ms'])
print(' '.join(out))")"
done
done
