#!/bin/bash
# Timing experiments on the sumcheck kernels with the development library (make BN_DEV=1):
# BN_SC_DBG (bit 0: synthetic operands instead of column loads, bit 1: no products, bit 2: no
# k-multiples, bit 3: no parity reduction), one
# kernel-trace per setting; results are wrong by design. Output: gpurun_out/scdbg_<n>/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp BINIUS_NTT_AMD_LIB="$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so"
cd /tmp
for n in ${SC_DBG_SET:-0 1 2 3}; do
  export BN_SC_DBG=$n
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/scdbg_$n" -o run -- python3 "$R/tools/bench_configs.py" --only c4 --sc-d ${SC_D:-3} > "$R/gpurun_out/scdbg_$n.log" 2>&1 || { echo "dbg $n failed"; tail -5 "$R/gpurun_out/scdbg_$n.log"; exit 1; }
  echo "== BN_SC_DBG=$n"; grep -h '"c4"' "$R/gpurun_out/scdbg_$n.log" | cut -c1-200
  f=$(find "$R/gpurun_out/scdbg_$n" -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | grep sc_ | sed 's/(bn::(anonymous namespace)::ScArgs)//'
  python3 "$R/tools/sc_round_gaps.py" "$R/gpurun_out/scdbg_$n/run_kernel_trace.csv" 24 > "$R/gpurun_out/scdbg_rounds_$n.txt" && head -1 "$R/gpurun_out/scdbg_rounds_$n.txt" && tail -6 "$R/gpurun_out/scdbg_rounds_$n.txt"
done
