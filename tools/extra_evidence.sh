#!/bin/bash
# Evidence beside tools/final_evidence.sh, into gpurun_out/profile_$ROUND_DIR/ (default r06):
#   sumcheck c4 d=3: rocprofv3 kernel trace + stats, per-round timeline, PMC (SQ and stall groups);
#   C3 (one 2^20 transform): kernel trace + stats of its three launches.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
P="$R/gpurun_out/profile_${ROUND_DIR:-r06}"
mkdir -p "$P"
export TMPDIR=/tmp
bash tools/prof_sumcheck.sh > /dev/null || exit 1
cp gpurun_out/prof_sc/run_kernel_stats.csv "$P/sumcheck_c4_d3_kernel_stats.csv"
python3 tools/sc_round_gaps.py gpurun_out/prof_sc/run_kernel_trace.csv 24 > "$P/sumcheck_c4_d3_rounds.txt" || exit 1
rm -rf gpurun_out/scpmc && mkdir -p gpurun_out/scpmc
PMC_GROUPS=sq,stall PMC_TAG=sc_ PMC_SCRIPT=tools/bench_configs.py PMC_ARGS="--only c4 --sc-d 3" bash tools/pmc.sh || exit 1
mv gpurun_out/pmc_sc_* gpurun_out/scpmc/
python3 tools/pmc_summary.py gpurun_out/scpmc > "$P/pmc_sumcheck_c4_d3.txt" || exit 1
c3() {  # tag, env...
  local tag=$1; shift
  ( cd /tmp && env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/c3_$tag" -o run -- python3 "$R/tools/bench_configs.py" --only c3 > "$R/gpurun_out/c3_$tag.log" 2>&1 ) || { echo "c3 $tag failed"; tail -5 "gpurun_out/c3_$tag.log"; return 1; }
  cp "gpurun_out/c3_$tag/run_kernel_stats.csv" "$P/c3_${tag}_kernel_stats.csv"
  grep -h '"c3"' "gpurun_out/c3_$tag.log" > "$P/c3_${tag}.json"
}
c3 default BN_NOTHING=1 || exit 1
echo "extra_evidence done"
