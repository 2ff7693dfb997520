#!/bin/bash
# A/B of the NTT kernel variants on one box: parity tests of the transform, then the headline
# bench (no CPU leg, no config-5 legs) once per variant. Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [[ -n "${AB_TESTS:-tests/test_gpu_ntt.py}" ]]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-300} python -u -m pytest ${AB_TESTS:-tests/test_gpu_ntt.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
for v in ${AB_VARIANTS:-1 5}; do
  timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 --variant $v > gpurun_out/ab_v$v.json 2> gpurun_out/ab_v$v.err || { echo "bench v$v failed rc=$?"; tail -20 gpurun_out/ab_v$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_v$v.json'));r=d['roofline'];print('variant $v: ms/step %.4f  passes %s  frac %.3f  transform_frac %.3f'%(d['ms_per_step'],['%.4f'%x for x in r['pass_ms']],r['frac'],r['transform_frac']))"
done
