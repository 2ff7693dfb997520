#!/bin/bash
# VERDICT r5 item 1 kill-test: strided 16-byte tile copy (binius-ntt_amd/tools/strided_copy.hip),
# timed, then FETCH_SIZE and WRITE_SIZE per variant in separate rocprofv3 passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
B="$R/binius-ntt_amd/devbin/strided_copy"
O="$R/gpurun_out/r06_kill"
mkdir -p "$O"
timeout -k 10 120 "$B" 20 > "$O/times.jsonl" 2>&1 && cat "$O/times.jsonl" \
 && timeout -k 10 120 "$B" 20 > "$O/times2.jsonl" 2>&1 && cat "$O/times2.jsonl" \
 && cd /tmp \
 && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d "$O/fetch" -o run -- "$B" 3 > "$O/fetch.log" 2>&1 \
 && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d "$O/write" -o run -- "$B" 3 > "$O/write.log" 2>&1 \
 && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d "$O/hit" -o run -- "$B" 3 > "$O/hit.log" 2>&1 \
 && echo killtest done
