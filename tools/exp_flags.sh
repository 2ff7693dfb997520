# Timing attribution for the NTT passes (results are wrong with any flag set): see BsParams::dbg.
set -o pipefail
for f in ${FLAGS:-0 1 3 4 7}; do
  echo "flags=$f"; BN_DEBUG_FLAGS=$f timeout -k 10 120 python bench.py --no-cpu --no-configs --steps 20 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline']['pass_ms'])" || exit 1
done
