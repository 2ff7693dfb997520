#!/bin/bash
# A/B of the lane-split NTT passes (dev build, BN_SPLIT=0/1) on the C3 2^20 transform, after the
# NTT parity tests on the product library. Each GPU step has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or north_star or c5 or variants" > gpurun_out/absplit_tests.log 2>&1 || { echo "ntt tests failed"; tail -40 gpurun_out/absplit_tests.log; exit 1; }
tail -1 gpurun_out/absplit_tests.log
export BINIUS_NTT_AMD_LIB=$R/binius-ntt_amd/lib-dev/libbinius_ntt_amd.so
for rep in 1 2; do
for s in 0 1; do
BN_SPLIT=$s timeout -k 10 200 python tools/bench_configs.py --only c3 > gpurun_out/absplit_$s.jsonl 2> gpurun_out/absplit.err || { echo "c3 failed"; tail -20 gpurun_out/absplit.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/absplit_$s.jsonl').readline());print('split=$s c3 ms %.4f'%d['ms'])"
done
done
BN_SPLIT=1 timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-configs --steps 10 --warmup 3 --log-h 20 > gpurun_out/absplit_bench.json 2> gpurun_out/absplit_bench.err || { echo "bench failed"; tail -20 gpurun_out/absplit_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/absplit_bench.json'));print('2^20 split passes', d['roofline']['pass_ms'], d['ms_per_step'])"
BN_SPLIT=0 timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-configs --steps 10 --warmup 3 --log-h 20 > gpurun_out/absplit_bench0.json 2> gpurun_out/absplit_bench.err || { echo "bench failed"; tail -20 gpurun_out/absplit_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/absplit_bench0.json'));print('2^20 unsplit passes', d['roofline']['pass_ms'], d['ms_per_step'])"
