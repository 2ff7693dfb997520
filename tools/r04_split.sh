#!/bin/bash
# Lane-split NTT passes: parity (NTT GPU tests), then the C3 (2^20) and headline lines.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt.py tests/test_fixtures.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { echo "ntt tests failed"; tail -40 gpurun_out/split_tests.log; exit 1; }
tail -1 gpurun_out/split_tests.log
for i in 1 2; do
timeout -k 10 200 python tools/bench_configs.py --only c3 > gpurun_out/split_c3_$i.jsonl 2> gpurun_out/split_c3.err || { echo "c3 failed"; tail -20 gpurun_out/split_c3.err; exit 1; }
cat gpurun_out/split_c3_$i.jsonl
done
timeout -k 10 300 python bench.py --no-cpu --no-c5 --no-configs --steps 20 --warmup 5 > gpurun_out/split_bench.json 2> gpurun_out/split_bench.err || { echo "bench failed"; tail -20 gpurun_out/split_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/split_bench.json'));print(d['ms_per_step'],d['roofline']['pass_ms'],d['config']['output_check'])"
