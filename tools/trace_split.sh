#!/bin/bash
# Per-phase cycles of the 2^20 NTT passes (dev build, BN_TRACE=1), lane-split (BN_SPLIT=1) vs one
# wave per limb (BN_SPLIT=0). -> gpurun_out/trace_split_*.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so BN_TRACE=1
for s in 0 1; do
BN_SPLIT=$s timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-configs --steps 2 --warmup 1 --log-h 20 > gpurun_out/trace_split_$s.json 2> gpurun_out/trace_split_$s.txt || { echo "trace failed"; tail -20 gpurun_out/trace_split_$s.txt; exit 1; }
echo "== BN_SPLIT=$s"; grep "trace pass" gpurun_out/trace_split_$s.txt | tail -3
done
