set -o pipefail
for lib in processing-chain_amd/pixpath/libpixpath.so tools/libvariants/siti_tilemajor.so processing-chain_amd/pixpath/libpixpath.so tools/libvariants/siti_tilemajor.so; do
  PIXPATH_LIB=$PWD/$lib timeout -k 10 150 python3 tools/siti_sizes.py || exit 1
done
