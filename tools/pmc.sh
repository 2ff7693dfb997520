#!/bin/bash
# PMC counter passes for the headline bench (each counter group in its own rocprofv3 run,
# kernel-trace only, as MI355X_MICROARCH.md prescribes). Output: gpurun_out/pmc_*/
# PMC_GROUPS selects passes (default: all); PMC_SCRIPT / PMC_ARGS select the profiled command
# (default: bench.py). Summarise with tools/pmc_summary.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
GROUPS_=${PMC_GROUPS:-fetch,write,sq,lds,ic}
run() {  # name, counters...
  local name=$1; shift
  [[ ",$GROUPS_," == *",$name,"* ]] || return 0
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -f csv -d "$R/gpurun_out/pmc_${PMC_TAG:-}$name" -o run -- python3 "$R/${PMC_SCRIPT:-bench.py}" ${PMC_ARGS:---no-cpu --no-configs --no-c5 --steps 3 --warmup 1} > "$R/gpurun_out/pmc_${PMC_TAG:-}$name.log" 2>&1 || { echo "pmc $name failed"; tail -5 "$R/gpurun_out/pmc_${PMC_TAG:-}$name.log"; return 1; }
}
run fetch FETCH_SIZE && run write WRITE_SIZE \
 && run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
 && run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
 && run stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
 && run ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
 && echo pmc done
