#!/bin/bash
# Builds and runs the reference's sumcheck benchmark driver on the C++ mirror
# (tools/cpp/benchmark_sumcheck.cpp); writes gpurun_out/benchmark_sumcheck.txt.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out tests/cpp/build
g++ -std=c++17 -O2 -I include -I binius-ntt_amd/host/ulvt tools/cpp/benchmark_sumcheck.cpp -o tests/cpp/build/benchmark_sumcheck \
  -L binius-ntt_amd/lib -lbinius_ntt_amd -Wl,-rpath,$R/binius-ntt_amd/lib -Wl,--allow-shlib-undefined || exit 1
timeout -k 10 600 tests/cpp/build/benchmark_sumcheck > gpurun_out/benchmark_sumcheck.txt 2>&1
rc=$?; cat gpurun_out/benchmark_sumcheck.txt; exit $rc
