# Build a variant of libbev_mi355x.so with extra compile definitions into tools/_ab/ (A/B timing only):
#   bash tools/build_variant.sh lines0 -DH16B_LINES=0
set -e
cd "$(dirname "$0")/../vision-based-spatio-temporal-analysis_amd"
name=$1; shift
out=../tools/_ab/$name; mkdir -p $out
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DBEV_SRC_HASH='"variant"' "$@" -c -o $out/$(basename $f .hip).o $f &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../tools/_ab/libbev_$name.so $out/*.o
rm -rf $out
