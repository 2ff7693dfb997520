#!/bin/bash
# A/B timing in one GPU session: CMD is run alternately with the in-tree library and with
# $ALT (a library built from another revision), REPS times each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
for i in $(seq ${REPS:-2}); do
  echo "== A (tree)"; timeout -k 10 300 bash -c "$CMD" || exit 1
  echo "== B ($ALT)"; BINIUS_NTT_AMD_LIB="$R/$ALT" timeout -k 10 300 bash -c "$CMD" || exit 1
done
