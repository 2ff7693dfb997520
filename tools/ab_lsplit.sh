#!/bin/bash
# One-limb single-wave work-groups for the GF(2^32) middle passes (dev build, BN_LSPLIT=1): GF(2^128)
# NTT parity tests with it on, then the headline passes with it off/on (two passes each).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
BN_LSPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gf128 or c5" > gpurun_out/abls_tests.log 2>&1 || { echo "ntt tests failed"; tail -40 gpurun_out/abls_tests.log; exit 1; }
tail -1 gpurun_out/abls_tests.log
for rep in 1 2; do
for s in 0 1; do
BN_LSPLIT=$s timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 > gpurun_out/abls_$s.json 2> gpurun_out/abls.err || { echo "bench failed"; tail -20 gpurun_out/abls.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/abls_$s.json'));print('lsplit=$s ms %.4f passes %s' % (d['ms_per_step'], ['%.4f'%x for x in d['roofline']['pass_ms']]))"
done
done
