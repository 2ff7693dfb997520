#!/bin/bash
# A/B of two builds of the library on one box (AB_LIBS = space-separated .so paths; "" = the
# in-tree product library): the NTT headline line and the c4 sumcheck lines for each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for L in ${AB_LIBS:-lib binius-ntt_amd/lib-x/libbinius_ntt_amd.so}; do
  i=$((i+1))
  if [[ $L == lib ]]; then unset BINIUS_NTT_AMD_LIB; else export BINIUS_NTT_AMD_LIB=$PWD/$L; fi
  echo "== $L"
  timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 > gpurun_out/ab$i.json 2> gpurun_out/ab$i.err || { echo "bench failed"; tail -5 gpurun_out/ab$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab$i.json'));print('ntt ms/step %.4f passes %s'%(d['ms_per_step'],['%.4f'%x for x in d['roofline']['pass_ms']]))"
  timeout -k 10 200 python tools/bench_configs.py --only ${AB_CONFIGS:-c4} --sc-d ${AB_SCD:-2,3,4} 2> gpurun_out/ab${i}_cfg.err | python3 -c "import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config'), d.get('workload','')[:60], 'ms %.3f'%d['ms'] if 'ms' in d else d)" || { echo "configs failed"; tail -5 gpurun_out/ab${i}_cfg.err; exit 1; }
done
