#!/bin/bash
# Round-4 evidence on one box, from the final library: the GPU suite, rocprofv3 kernel stats of the
# headline bench, PMC passes (headline + config 2) -> gpurun_out/pmc_kernels.json (bench.py's
# PMC_FILE), config 3 (2^20) kernel stats + PMC, the default bench line, the c4 sumcheck timeline.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out && rm -rf gpurun_out/pmc_* gpurun_out/prof gpurun_out/c3pmc gpurun_out/c3prof
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -s > gpurun_out/r04f_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r04f_tests.log; exit 1; }
tail -1 gpurun_out/r04f_tests.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-configs --no-c5 --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1 ) || { echo "rocprof headline failed"; tail -20 gpurun_out/prof.log; exit 1; }
PMC_GROUPS=fetch,write,sq,stall,lds bash tools/pmc.sh || exit 1
PMC_TAG=c2_ PMC_GROUPS=sq PMC_SCRIPT=tools/bench_configs.py PMC_ARGS="--only c2" bash tools/pmc.sh || exit 1
python3 tools/pmc_summary.py --traffic 24 > gpurun_out/pmc_summary.txt || exit 1
python3 tools/pmc_summary.py --kernels gpurun_out/pmc_kernels.json "round-4 final library: bench.py headline passes (fetch, write, sq, stall, lds) + config-2 kernels (sq)" > /dev/null || exit 1
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/c3prof" -o run -- python3 "$R/tools/bench_configs.py" --only c3 > "$R/gpurun_out/c3prof.log" 2>&1 ) || { echo "rocprof c3 failed"; exit 1; }
for g in "sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" "fetch FETCH_SIZE" "write WRITE_SIZE"; do
  set -- $g; name=$1; shift
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -f csv -d "$R/gpurun_out/c3pmc/pmc_$name" -o run -- python3 "$R/tools/bench_configs.py" --only c3 > "$R/gpurun_out/c3pmc_$name.log" 2>&1 ) || { echo "c3 pmc $name failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/c3pmc > gpurun_out/c3pmc_summary.txt || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { echo "bench failed"; tail -20 gpurun_out/r04f_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04f_bench.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['pass_ms'],[(c['config'],c.get('ms')) for c in d['configs']])"
bash tools/sc_trace.sh > /dev/null || exit 1
head -1 gpurun_out/sc_rounds.txt
echo "r04 final done"
