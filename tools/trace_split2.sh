#!/bin/bash
# Lane-split 2^20 passes with and without the scheduling barriers around the products (dev builds
# lib-dev / lib-dx, BN_SPLIT=1 BN_TRACE=1): per-phase cycles and the C3 time.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
for L in lib-dev; do
export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/$L/libbinius_ntt_amd.so
BN_TRACE=1 BN_SPLIT=1 timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-configs --steps 2 --warmup 1 --log-h 20 > gpurun_out/ts2_$L.json 2> gpurun_out/ts2_$L.txt || { echo "trace failed"; tail -20 gpurun_out/ts2_$L.txt; exit 1; }
echo "== $L"; grep "trace pass" gpurun_out/ts2_$L.txt | tail -2
BN_SPLIT=1 timeout -k 10 200 python tools/bench_configs.py --only c3 > gpurun_out/ts2_c3_$L.jsonl 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/ts2_c3_$L.jsonl').readline());print('c3 ms %.4f'%d['ms'])"
done
