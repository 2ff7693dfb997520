#!/bin/bash
# One GPU session that regenerates the committed evidence for the headline NTT: rocprofv3 kernel
# stats of bench.py, PMC passes (one counter group per run), the HBM-traffic summary read by
# bench.py, and a full bench line (with the CPU baseline). Outputs under gpurun_out/; copy the
# ones to keep into profiles/<round>/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out && rm -rf gpurun_out/prof gpurun_out/pmc_*
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-configs --no-c5 --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1 ) || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
PMC_GROUPS=${PMC_GROUPS:-fetch,write,sq,stall,lds} bash tools/pmc.sh || exit 1
python3 tools/pmc_summary.py --traffic 24 > gpurun_out/pmc_summary.txt || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo refresh done
