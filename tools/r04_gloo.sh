#!/bin/bash
# bench.py at world size 2 over gloo on one GPU (both ranks share the card): the multi-rank path
# of the driver's N > 1 runs, incl. the sharded sumcheck's per-round exchange. -> gpurun_out/bench_gloo2.json
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
BENCH_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --no-cpu --no-configs --steps 10 --warmup 3 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo "gloo bench failed"; tail -30 gpurun_out/bench_gloo2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_gloo2.json'));print(d['n_gpus'], d['ms_per_step'], json.dumps(d['c5']['sumcheck']))"
