#!/bin/bash
# usage: tools/resources.sh <file.hip> [filter]  -- per-kernel VGPR / spill / occupancy summary
f=$1; filt=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c -o /tmp/_res.o "$f" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/\[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/{n=$NF} /VGPRs:/{v=$NF} /SGPRs Spill/{ss=$NF} /VGPRs Spill/{vs=$NF} /Occupancy/{o=$NF}
       /LDS Size/{print n, "vgpr="v, "occ="o, "sspill="ss, "vspill="vs, "lds="$NF}' | grep -E "$filt"
