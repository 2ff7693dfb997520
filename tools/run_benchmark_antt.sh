#!/bin/bash
# Builds and runs the benchmark_antt-format harness (tools/cpp/benchmark_antt.cpp) on the GPU;
# writes gpurun_out/benchmark_antt.txt.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out tests/cpp/build
python3 -c "import json; h=json.load(open('tests/golden/additive_ntt_md5.json'))['hashes']['0']; open('gpurun_out/hashes_r0.txt','w').write(''.join('%d %s\n'%(i,x) for i,x in enumerate(h) if x))"
g++ -std=c++17 -O2 -I include -I binius-ntt_amd/host/ulvt tools/cpp/benchmark_antt.cpp -o tests/cpp/build/benchmark_antt \
  -L binius-ntt_amd/lib -lbinius_ntt_amd -L oracle -loracle -Wl,-rpath,$R/binius-ntt_amd/lib -Wl,-rpath,$R/oracle -Wl,--allow-shlib-undefined
timeout -k 10 600 tests/cpp/build/benchmark_antt gpurun_out/hashes_r0.txt ${MAX_LOG_H:-28} > gpurun_out/benchmark_antt.txt 2>&1
rc=$?; cat gpurun_out/benchmark_antt.txt; exit $rc
