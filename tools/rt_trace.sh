#!/bin/bash
# Dev helper: register-tile (variant 4) phase trace and the no-load / no-store timings, on the
# development library (make -C binius-ntt_amd BN_DEV=1). Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BINIUS_NTT_AMD_LIB=$PWD/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
BN_TRACE=1 timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 1 --warmup 1 --variant ${RT_VARIANT:-4} > gpurun_out/rt_trace.json 2> gpurun_out/rt_trace.err || { tail -5 gpurun_out/rt_trace.err; exit 1; }
grep "^trace" gpurun_out/rt_trace.err | tail -3
for f in 0 1 2 3; do
  BN_DEBUG_FLAGS=$f timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 10 --warmup 2 --variant ${RT_VARIANT:-4} > gpurun_out/rt_dbg$f.json 2> gpurun_out/rt_dbg$f.err || { tail -5 gpurun_out/rt_dbg$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/rt_dbg$f.json'));print('dbg $f: ms/step %.4f passes %s'%(d['ms_per_step'],['%.4f'%x for x in d['roofline']['pass_ms']]))"
done
