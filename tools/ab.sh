#!/bin/bash
# A/B timing in one GPU session: CMD is run alternately with the in-tree library and with each
# library in $ALT (space-separated, built from other revisions), REPS rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
for i in $(seq ${REPS:-2}); do
  echo "== tree"; timeout -k 10 300 bash -c "$CMD" || exit 1
  for a in $ALT; do
    echo "== $a"; BINIUS_NTT_AMD_LIB="$R/$a" timeout -k 10 300 bash -c "$CMD" || exit 1
  done
done
