# Build a strip-kernel library variant with extra -D flags into tools/var/libpixpath_<name>.so
# (the scaler units recompiled with the flags; every other object is the product's).
# usage: bash tools/build_var_r6.sh <name> "-DFOO=1"
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../processing-chain_amd"
out=build/var_$name; mkdir -p $out ../tools/var
for f in scale.hip strip_u16.hip strip_u16_chain.hip strip_u8.hip strip_u8_chain.hip strip_u16_fused.hip strip_u8_fused.hip siti.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result $defs -x hip -c csrc/$f -o $out/$f.o &
done
wait
objs=$(ls build/*.o | grep -v -E "scale.hip|strip_u16|strip_u8|siti.hip")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/var/libpixpath_$name.so $objs $out/*.o
echo built tools/var/libpixpath_$name.so
