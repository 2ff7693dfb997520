#!/bin/bash
# Multi-rank paths after a change: the distributed GPU tests (gloo world 2, incl. the staged device
# exchange; RCCL world 1), bench.py at world 1 and over gloo at world 2 (c5 legs present, no error).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_gpu_rccl_world1.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { echo "dist tests failed"; tail -30 gpurun_out/dist_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/dist_tests.log | tail -1
timeout -k 10 300 python bench.py --no-cpu --no-configs --steps 5 --warmup 2 > gpurun_out/dc_w1.json 2> gpurun_out/dc_w1.err || { echo "bench w1 failed"; tail -20 gpurun_out/dc_w1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/dc_w1.json'));print('w1', d['ms_per_step'], d['c5']['sumcheck'].get('error'), d['c5']['sumcheck'].get('ms'))"
BENCH_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --no-cpu --no-configs --steps 5 --warmup 2 > gpurun_out/dc_w2.json 2> gpurun_out/dc_w2.err || { echo "bench w2 failed"; tail -20 gpurun_out/dc_w2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/dc_w2.json'));print('w2', d['ms_per_step'], d['c5']['sumcheck'].get('error'), d['c5']['sumcheck'].get('ms'), d['c5']['sumcheck'].get('exchange_ms_per_round'))"
