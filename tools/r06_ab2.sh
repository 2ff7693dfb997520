#!/bin/bash
# Round-6 A/Bs on one box, after their parity tests:
#  1. VERDICT r5 item 2: the big rounds' fold fused into the next round's messages (sc_fold_msgs,
#     product library) against separate fold + messages launches (lib-nf, -DBN_SC_NO_FUSED):
#     the sumcheck GPU tests first, then c4 d = 2, 3, 4, three alternating pairs;
#  2. VERDICT r5 item 5: 2^24 NTT as 7 + 6 + 11 stages (dev build, BN_BOTTOM_K=11) against
#     7 + 5 + 12, three alternating pairs, after its parity tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r06_ab2
mkdir -p $O
unset BINIUS_NTT_AMD_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_sumcheck_large.py -m gpu > $O/parity_fused.txt 2>&1 \
  || { echo "sumcheck parity failed"; tail -30 $O/parity_fused.txt; exit 1; }
tail -2 $O/parity_fused.txt
c4() {  # tag, [library]
  local T=$1 L=${2:-}
  (if [[ -n $L ]]; then export BINIUS_NTT_AMD_LIB=$L; else unset BINIUS_NTT_AMD_LIB; fi && timeout -k 10 240 python tools/bench_configs.py --only c4 --sc-d 2,3,4 2> "$R/$O/c4_$T.err") \
   | python3 -c "import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l)
        if 'bitsliced' in d.get('workload',''): print('$T', d.get('workload','')[:60], 'ms %.3f'%d['ms'])"
}
for rep in 1 2 3; do
  c4 fused || exit 1
  c4 separate "$R/binius-ntt_amd/lib-nf/libbinius_ntt_amd.so" || exit 1
done
export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
BN_BOTTOM_K=11 BN_RR_LAST=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ntt.py \
  -m gpu -k "not register_tile and not variant and not lane_split and (gf32_r0_reference_md5 or gf128_matches_oracle or north_star_size or gf128_batched or c5_batched or 2p26)" > $O/parity_bottom11.txt 2>&1 \
  || { echo "ntt parity failed"; tail -20 $O/parity_bottom11.txt; exit 1; }
tail -2 $O/parity_bottom11.txt
for rep in 1 2 3; do
  for K in 12 11; do
    BN_BOTTOM_K=$K timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 > $O/ntt_k${K}_$rep.json 2> $O/ntt_k${K}_$rep.err || { echo "bench failed"; tail -5 $O/ntt_k${K}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ntt_k${K}_$rep.json'));print('bottom_k $K ms/step %.4f passes %s'%(d['ms_per_step'],['%.4f'%x for x in d['roofline']['pass_ms']]))"
  done
done
echo ab2 done
