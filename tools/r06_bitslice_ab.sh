#!/bin/bash
# Round 6: bn_bitslice_device on LDS-staged coalesced waves against the previous library's
# one-thread-per-block kernel (abr/old = git worktree of the previous commit, built in place).
# Parity first (field + sumcheck tests, which construct provers from compact input), then both
# directions on 2^20 blocks (512 MiB in place) and the compact-input sumcheck phases (c4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[[ -n $SKIP_PARITY ]] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_field.py \
  tests/test_gpu_sumcheck.py tests/test_fixtures.py > gpurun_out/bitslice_parity.txt 2>&1 || { tail -30 gpurun_out/bitslice_parity.txt; exit 1; }
echo "parity: $(tail -1 gpurun_out/bitslice_parity.txt)"
for rep in 1 2; do
  for L in old new; do
    if [[ $L == old ]]; then export BINIUS_NTT_AMD_LIB=$PWD/abr/old/binius-ntt_amd/lib/libbinius_ntt_amd.so; else unset BINIUS_NTT_AMD_LIB; fi
    echo "== $L"
    PYTHONPATH=$PWD/binius-ntt_amd/python timeout -k 10 120 python - <<'PY' || exit 1
import torch, binius_ntt_amd as B
dev = torch.device("cuda:0"); st = torch.cuda.current_stream(dev)
x = torch.randint(-2**31, 2**31, (128 << 20,), dtype=torch.int32, device=dev)
for unt in (0, 1):
    for _ in range(2): B.bitslice(x, untranspose=bool(unt))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(10): B.bitslice(x, untranspose=bool(unt))
    b.record(st); b.synchronize()
    ms = a.elapsed_time(b) / 10
    print("bitslice untranspose=%d: %.4f ms, %.0f GB/s (512 MiB read + written)" % (unt, ms, 2 * 2**29 / (ms * 1e-3) / 1e9))
PY
    timeout -k 10 400 python tools/bench_configs.py --only c4 --sc-d 3 2>/dev/null | grep "compact input" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:40], 'transpose_ms %.3f raw_ms %.3f' % (d['transpose_ms'], d['raw_ms']))" || exit 1
  done
done
