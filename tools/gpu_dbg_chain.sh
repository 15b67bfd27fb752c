set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/dbg_chain.py || exit 1
TAG=noclamp PIXPATH_LIB=$PWD/tools/ablate/libpixpath_noclamp.so timeout -k 10 120 python3 tools/dbg_chain.py || exit 1
TAG=r3 PIXPATH_LIB=$PWD/tools/ablate/libpixpath_r3.so timeout -k 10 120 python3 tools/dbg_chain.py || exit 1
