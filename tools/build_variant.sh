# Build a library variant with extra -D flags into tools/ablate/libpixpath_<name>.so
# (only the scaler sources are recompiled; the rest are the product objects).
# usage: bash tools/build_variant.sh <name> "-DFOO -DBAR=3"
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../processing-chain_amd"
out=build/var_$name; mkdir -p $out ../tools/ablate
for f in scale.hip strip_u16.hip strip_u16_chain.hip strip_u8.hip strip_u8_chain.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result $defs -x hip -c csrc/$f -o $out/$f.o &
done
wait
objs=$(ls build/*.o | grep -v -E "scale.hip|strip_u16|strip_u8")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/ablate/libpixpath_$name.so $objs $out/*.o
echo built tools/ablate/libpixpath_$name.so
