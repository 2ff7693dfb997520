#!/bin/bash
# VERDICT r5 item 2 evidence: per-round kernel timelines of c4 d = 3 (rocprofv3 kernel trace ->
# tools/sc_round_gaps.py) with the big rounds' fold fused into the messages launch (lib-fu,
# -DBN_SC_FUSED) and with separate launches (the product library), then the fused kernel's PMC
# (FETCH_SIZE, WRITE_SIZE, the SQ stall group), each pass in its own rocprofv3 run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r06_fused
mkdir -p $O
export TMPDIR=/tmp
trace() {  # tag, library
  local T=$1 L=$2
  ( cd /tmp && BINIUS_NTT_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$R/$O/tr_$T" -o run -- python3 "$R/tools/bench_configs.py" --only c4 --sc-d 3 > "$R/$O/tr_$T.log" 2>&1 ) || { echo "trace $T failed"; tail -5 $O/tr_$T.log; return 1; }
  python3 tools/sc_round_gaps.py $O/tr_$T/run_kernel_trace.csv 24 > $O/rounds_$T.txt && head -12 $O/rounds_$T.txt
}
trace fused "$R/binius-ntt_amd/lib-fu/libbinius_ntt_amd.so" && trace separate "$R/binius-ntt_amd/lib/libbinius_ntt_amd.so" || exit 1
export BINIUS_NTT_AMD_LIB="$R/binius-ntt_amd/lib-fu/libbinius_ntt_amd.so"
PMC_GROUPS=fetch,write,stall PMC_TAG=fu_ PMC_SCRIPT=tools/bench_configs.py PMC_ARGS="--only c4 --sc-d 3" bash tools/pmc.sh || exit 1
unset BINIUS_NTT_AMD_LIB
PMC_GROUPS=fetch,write,stall PMC_TAG=sep_ PMC_SCRIPT=tools/bench_configs.py PMC_ARGS="--only c4 --sc-d 3" bash tools/pmc.sh || exit 1
mkdir -p $O/pmc_fu $O/pmc_sep && mv gpurun_out/pmc_fu_* $O/pmc_fu/ && mv gpurun_out/pmc_sep_* $O/pmc_sep/
python3 tools/pmc_summary.py $O/pmc_fu > $O/pmc_fused.txt && python3 tools/pmc_summary.py $O/pmc_sep > $O/pmc_separate.txt && echo fused_prof done
