#!/bin/bash
# Per-round c4 timelines (tools/sc_trace.sh) for several builds of the library:
# AB_LIBS = space-separated .so paths ("lib" = the in-tree product library);
# gpurun_out/sc_rounds_<i>.txt for each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
i=0
for L in ${AB_LIBS:-lib}; do
  i=$((i+1))
  if [[ $L == lib ]]; then unset BINIUS_NTT_AMD_LIB; else export BINIUS_NTT_AMD_LIB=$R/$L; fi
  echo "== $L"
  "$R/tools/sc_trace.sh" > /dev/null || exit 1
  cp "$R/gpurun_out/sc_rounds.txt" "$R/gpurun_out/sc_rounds_$i.txt"
  cat "$R/gpurun_out/sc_rounds_$i.txt"
done
