#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) of the c4 d=3 sumcheck for the
# round-3 library (lib-base) and the current one: instruction mix, wait and LDS counters of the
# big-round kernels. -> gpurun_out/scpmc_{base,cur}/pmc_*/, summaries in gpurun_out/scpmc_*.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
for L in base cur; do
  if [[ $L == base ]]; then export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-base/libbinius_ntt_amd.so; else unset BINIUS_NTT_AMD_LIB; fi
  run() {  # group name, counters...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -f csv -d "$R/gpurun_out/scpmc_$L/pmc_$name" -o run -- python3 "$R/tools/bench_configs.py" --only c4 --sc-d 3 > "$R/gpurun_out/scpmc_${L}_$name.log" 2>&1 || { echo "pmc $L $name failed"; tail -5 "$R/gpurun_out/scpmc_${L}_$name.log"; return 1; }
  }
  run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
  run stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT || exit 1
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/scpmc_$L" > "$R/gpurun_out/scpmc_$L.txt" 2>&1 || exit 1
  echo "== $L"; grep -A20 "sc_messages<0, 4>\|sc_fold_coal" "$R/gpurun_out/scpmc_$L.txt" | head -40
done
