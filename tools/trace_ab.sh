#!/bin/bash
# Dev helper: per-wave phase trace (BN_TRACE) + short bench for each env setting in $VARIANTS
# (";"-separated, e.g. VARIANTS="BN_PF=0;BN_PF=1").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -ra VS <<< "${VARIANTS:-BN_PF=1}"
for v in "${VS[@]}"; do
  echo "== $v"
  env $v BN_TRACE=1 timeout -k 10 120 python bench.py --no-cpu --no-configs --steps 1 --warmup 1 > gpurun_out/trace.json 2> gpurun_out/trace.err || { tail -5 gpurun_out/trace.err; exit 1; }
  grep "^trace" gpurun_out/trace.err | tail -3
  env $v bash tools/bench_brief.sh || exit 1
done
