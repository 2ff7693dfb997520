#!/bin/bash
# Round-6 A/Bs on one box:
#  1. VERDICT r5 item 3: sumcheck c4 (d = 2, 3, 4) of the round-4 library (abr/r04, git de2596f,
#     built from its own tree) against the current one, three alternating pairs; also the current
#     library built with 128-thread sumcheck work-groups (lib-t128, -DBN_SC_THREADS=128);
#  2. VERDICT r5 item 5: 2^24 NTT as 7 + 6 + 11 stages (dev build, BN_BOTTOM_K=11) against
#     7 + 5 + 12, three alternating pairs, after its parity tests.
# (setup, in the container: mkdir -p abr/r04 && git archive de2596f | tar -x -C abr/r04 &&
#  make -C abr/r04/binius-ntt_amd ARCH=gfx950; abr/ is git-ignored)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r06_ab1
mkdir -p $O
c4() {  # tag, tree, [library]
  local T=$1 D=$2 L=${3:-}
  (cd "$D" && if [[ -n $L ]]; then export BINIUS_NTT_AMD_LIB=$L; else unset BINIUS_NTT_AMD_LIB; fi && timeout -k 10 240 python tools/bench_configs.py --only c4 --sc-d 2,3,4 2> "$R/$O/c4_$T.err") \
   | python3 -c "import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('$T', d.get('config'), d.get('workload','')[:70], 'ms %.3f'%d['ms'] if 'ms' in d else d)"
}
for rep in 1 2 3; do
  c4 r04 "$R/abr/r04" || exit 1
  c4 cur "$R" || exit 1
  c4 t128 "$R" "$R/binius-ntt_amd/lib-t128/libbinius_ntt_amd.so" || exit 1
done
export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
BN_BOTTOM_K=11 BN_RR_LAST=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ntt.py \
  -m gpu -k "gf32_r0_reference_md5 or gf128_matches_oracle or north_star_size or gf128_batched or c5_batched or 2p26" > $O/parity_bottom11.txt 2>&1 \
  || { echo "parity failed"; tail -20 $O/parity_bottom11.txt; exit 1; }
tail -2 $O/parity_bottom11.txt
for rep in 1 2 3; do
  for K in 12 11; do
    BN_BOTTOM_K=$K timeout -k 10 120 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 3 > $O/ntt_k${K}_$rep.json 2> $O/ntt_k${K}_$rep.err || { echo "bench failed"; tail -5 $O/ntt_k${K}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ntt_k${K}_$rep.json'));print('bottom_k $K ms/step %.4f passes %s'%(d['ms_per_step'],['%.4f'%x for x in d['roofline']['pass_ms']]))"
  done
done
echo ab1 done
