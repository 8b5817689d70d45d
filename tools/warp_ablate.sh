# Build timing-only variants of the fused warp (bev_warp.hip with -DWARP_ABLATE=<bits>) into tools/_ablate/.
# Run here (hipcc cross-compiles); tools/warp_ablate.py times them on the GPU.  Never the product library.
set -eu
cd "$(dirname "$0")/.."
SRC=vision-based-spatio-temporal-analysis_amd/csrc/bev_warp.hip
for b in ${@:-0 1 2 4 8 16 12 18}; do  # WARP_ABLATE bits (WARP_OPT via OPT env)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -shared -DWARP_ABLATE=$b -DWARP_OPT=${OPT:-1} ${EXTRA:-} \
    -o tools/_ablate/libwarp_ablate_${b}${SUF:-}.so $SRC &
done
wait
