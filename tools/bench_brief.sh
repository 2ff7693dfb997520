#!/bin/bash
# One short headline bench, printed as "ms_per_step [pass ms...]" (A/B helper for tools/dbg_flags_ab.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 120 python bench.py --no-cpu --no-configs --steps ${STEPS:-20} ${BENCH_ARGS:-} | python3 -c "import json,sys; d=json.load(sys.stdin); print('%.4f' % d['ms_per_step'], ['%.4f' % x for x in d['roofline']['pass_ms']])"
