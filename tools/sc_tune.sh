#!/bin/bash
# Threshold sweep for the sumcheck launch choices with the development library (make BN_DEV=1):
# SC_TUNE = space-separated HEX_MAX:POST_MAX[:WIDE_MAX] settings; c4 lines for each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export BINIUS_NTT_AMD_LIB="$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so"
for hp in ${SC_TUNE:-8192:64}; do
  IFS=: read -r hx px wx <<< "$hp"
  export BN_SC_HEX_MAX=$hx BN_SC_POST_MAX=$px BN_SC_WIDE_MAX=${wx:-1024}
  echo "== hex_max $BN_SC_HEX_MAX post_max $BN_SC_POST_MAX wide_max $BN_SC_WIDE_MAX"
  timeout -k 10 200 python tools/bench_configs.py --only c4 --sc-d ${SC_D:-2,3,4} 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l)
        if 'ms' in d: print(d['workload'][-30:], 'ms %.3f'%d['ms'])" || { echo "c4 failed"; exit 1; }
done
