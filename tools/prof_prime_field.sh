#!/bin/bash
# Prime-field siblings on one GPU box: parity tests, bench lines, rocprofv3 kernel stats.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_qm31_sumcheck.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/qm_t.log 2>&1
timeout -k 10 200 python -u tools/bench_configs.py --only qm,bb > gpurun_out/qm_b.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_pf -o pf -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --only qm,bb > $GRAFT_REPO_ROOT/gpurun_out/prof_pf.log 2>&1
