#!/bin/bash
# Round-6 check that the product sumcheck is round 5's again (the round-6 refactor of sc_fold_pair
# into a per-item helper had made round 0's fold 316 -> 420-428 us): sumcheck GPU tests on the
# product library and on the fused experiment build (lib-fu), then c4 d = 2, 3, 4 of the round-5
# library (abr/r05, git 979a509, built from its own tree) against the current one, three
# alternating pairs, and the per-round timelines of both.
# (setup, in the container: mkdir -p abr/r05 && git archive 979a509 | tar -x -C abr/r05 &&
#  make -C abr/r05/binius-ntt_amd ARCH=gfx950; abr/ is git-ignored)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r06_ab3
mkdir -p $O
unset BINIUS_NTT_AMD_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py tests/test_distributed.py -m gpu > $O/parity_product.txt 2>&1 \
  || { echo "product parity failed"; tail -30 $O/parity_product.txt; exit 1; }
tail -1 $O/parity_product.txt
BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-fu/libbinius_ntt_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py -m gpu > $O/parity_fused.txt 2>&1 \
  || { echo "fused parity failed"; tail -30 $O/parity_fused.txt; exit 1; }
tail -1 $O/parity_fused.txt
c4() {  # tag, tree
  local T=$1 D=$2
  (cd "$D" && timeout -k 10 240 python tools/bench_configs.py --only c4 --sc-d 2,3,4 2> "$R/$O/c4_$T.err") \
   | python3 -c "import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l)
        if 'bitsliced' in d.get('workload',''): print('$T', d.get('workload','')[:60], 'ms %.3f'%d['ms'])"
}
for rep in 1 2 3; do
  c4 r05 "$R/abr/r05" || exit 1
  c4 r06 "$R" || exit 1
done
export TMPDIR=/tmp
for T in r05 r06; do
  D="$R"; [[ $T == r05 ]] && D="$R/abr/r05"
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$R/$O/tr_$T" -o run -- python3 "$D/tools/bench_configs.py" --only c4 --sc-d 3 > "$R/$O/tr_$T.log" 2>&1 ) || { echo "trace $T failed"; exit 1; }
  python3 tools/sc_round_gaps.py $O/tr_$T/run_kernel_trace.csv 24 > $O/rounds_$T.txt && head -8 $O/rounds_$T.txt
done
echo ab3 done
