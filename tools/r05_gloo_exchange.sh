#!/bin/bash
# gloo world 2 on one GPU: bench.py's config-5 sumcheck with the host-staged and the device-sink
# exchange, alternated twice -> gpurun_out/gx_<path>_<rep>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for x in host device; do
    BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu --no-configs --steps 5 --warmup 2 --sc-exchange $x > gpurun_out/gx_${x}_$rep.json 2> gpurun_out/gx_${x}_$rep.err || { tail -20 gpurun_out/gx_${x}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['c5']['sumcheck']; print(sys.argv[2], s['exchange_path'], 'ms %.2f' % s['ms'], 'exchange/round %.4f' % s['exchange_ms_per_round'], 'messages/round %.4f' % s['messages_ms_per_round'])" gpurun_out/gx_${x}_$rep.json $x
  done
done
