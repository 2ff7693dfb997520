#!/bin/bash
# rocprofv3 kernel stats and PMC passes of the headline transform alone (bench.py without the c5 legs, whose batched launches
# share the pass kernels' names) + config 2 -> gpurun_out/pmc_kernels.json, gpurun_out/pmc_summary.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out && rm -rf gpurun_out/pmc_* gpurun_out/prof
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-configs --no-c5 --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1 ) || { echo "rocprof headline failed"; tail -20 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log | cut -c1-300
PMC_GROUPS=fetch,write,sq,stall,lds bash tools/pmc.sh || exit 1
PMC_TAG=c2_ PMC_GROUPS=sq PMC_SCRIPT=tools/bench_configs.py PMC_ARGS="--only c2" bash tools/pmc.sh || exit 1
python3 tools/pmc_summary.py --traffic 24 > gpurun_out/pmc_summary.txt || exit 1
python3 tools/pmc_summary.py --kernels gpurun_out/pmc_kernels.json "round-4 final library: bench.py headline passes without the c5 legs (fetch, write, sq, stall, lds) + config-2 kernels (sq)" > /dev/null || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/pmc_kernels.json'))
for k,v in d['kernels'].items():
    if 'antt' in k: print(k[:48], 'VALU %.4g waves %.4g HBM %.4g' % (v.get('SQ_INSTS_VALU',0), v.get('SQ_WAVES',0), v.get('HBM_BYTES',0)))
"
