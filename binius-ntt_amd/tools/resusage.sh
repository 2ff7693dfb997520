#!/bin/bash
# Print per-kernel VGPR / spill / occupancy for one HIP source (dev tool).
f=${1:-csrc/antt_bs.hip}
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I"$(dirname "$0")/../../include" -c "$f" -o /tmp/resusage.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep remark | sed 's/.*remark: //; s/ \[-Rpass.*//' |
  awk '/Function Name/{name=$3} /VGPRs:/{v=$2} /VGPRs Spill/{sp=$3} /Occupancy/{o=$3} /LDS Size/{print name, "vgpr=" v, "spill=" sp, "occ=" o}'
