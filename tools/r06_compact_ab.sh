#!/bin/bash
# Round 6: compact GF(2^128) elementwise products (bn_gf128_mul_device) on the quad-lane bitsliced
# product, and the sentinel-log GF(2^8) leaves of the compact kernels, against the previous library (abr/old = a worktree of the
# previous commit, built in place: git worktree add abr/old <rev> && make -C abr/old/binius-ntt_amd).
# Parity first (the GPU suite: field KATs, fixtures, the NTT MD5 tables through antt_v0_group), then the config-2 lines of both libraries on this box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${AB_TESTS:-tests} > gpurun_out/compact_parity.txt 2>&1 || { tail -30 gpurun_out/compact_parity.txt; exit 1; }
tail -3 gpurun_out/compact_parity.txt
for rep in 1 2; do
  for L in old new; do
    if [[ $L == old ]]; then export BINIUS_NTT_AMD_LIB=$PWD/abr/old/binius-ntt_amd/lib/libbinius_ntt_amd.so; else unset BINIUS_NTT_AMD_LIB; fi
    echo "== $L rep $rep"
    timeout -k 10 200 python tools/bench_configs.py --only c2 2> gpurun_out/compact_ab_$L.err | grep -E '"c2"' || { tail -5 gpurun_out/compact_ab_$L.err; exit 1; }
  done
done
