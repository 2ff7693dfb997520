#!/bin/bash
# Quick NTT A/B on one box: bench lines (no CPU / config-5 / configs legs) for each entry of
# AB_RUNS ("name:ENV=VAL,ENV=VAL:bench-args"), each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [[ -n "${AB_TESTS:-}" ]]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-300} python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abq_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/abq_pytest.log; exit 1; }
  tail -2 gpurun_out/abq_pytest.log
fi
IFS=';' read -ra RUNS <<< "${AB_RUNS}"
for run in "${RUNS[@]}"; do
  name=${run%%:*}; rest=${run#*:}; envs=${rest%%:*}; args=${rest#*:}
  ( IFS=','; for e in $envs; do [[ -n $e ]] && export "$e"; done; IFS=' '
    timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 $args > gpurun_out/abq_$name.json 2> gpurun_out/abq_$name.err ) || { echo "bench $name failed rc=$?"; tail -20 gpurun_out/abq_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abq_$name.json'));r=d['roofline'];print('$name: ms/step %.4f  passes %s  frac %.3f  transform_frac %.3f'%(d['ms_per_step'],['%.4f'%x for x in r['pass_ms']],r['frac'],r['transform_frac']))"
done
