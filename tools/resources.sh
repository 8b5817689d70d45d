#!/bin/bash
# usage: tools/resources.sh <file.hip> [filter]  -- per-kernel VGPR / scratch (private segment) / LDS summary
# (the code-object metadata lists a kernel's LDS size before its .name and its register counts after it)
f=$(realpath "$1"); filt=${2:-.}
d=$(mktemp -d)
(cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c -save-temps -o k.o "$f" 2>/dev/null)
s=$(ls $d/*gfx950*.s 2>/dev/null | head -1)
if [ -z "$s" ]; then echo "compile failed"; rm -rf $d; exit 1; fi
grep -E "^\s+\.(name|private_segment_fixed_size|vgpr_count|vgpr_spill_count|group_segment_fixed_size):" "$s" |
  awk '/\.name:/{if(n!="")print n, "vgpr="v, "scratch="p, "spill="sp, "lds="g; n=$2; g=gp} /private_segment/{p=$2} /vgpr_count/{v=$2} /vgpr_spill/{sp=$2} /group_segment/{gp=$2} END{print n, "vgpr="v, "scratch="p, "spill="sp, "lds="g}' |
  grep -E "$filt" | sed 's/_ZN12_GLOBAL__N_1[0-9]*//'
rm -rf $d
