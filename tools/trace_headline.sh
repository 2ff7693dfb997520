#!/bin/bash
# Per-phase cycles per wave-tile of the 2^24 passes (dev build, BN_TRACE=1). -> gpurun_out/trace_hl.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so BN_TRACE=1 timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-configs --steps 2 --warmup 1 > gpurun_out/trace_hl.json 2> gpurun_out/trace_hl.txt || { echo "trace failed"; tail -20 gpurun_out/trace_hl.txt; exit 1; }
grep "trace pass" gpurun_out/trace_hl.txt | tail -3
