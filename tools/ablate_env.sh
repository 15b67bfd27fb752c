# Sourced by the ablation / tuning scripts: they need the measurement build of
# the library (PIXPATH_* knobs compiled in; csrc/common.hpp PP_KNOB), built on
# the CPU before the gpurun call:  make -C processing-chain_amd ablate
ABL=$PWD/tools/ablate/libpixpath_ablate.so
[ -f "$ABL" ] || { echo "tools/ablate/libpixpath_ablate.so missing: make -C processing-chain_amd ablate"; exit 1; }
export PIXPATH_LIB=$ABL
BENCH_TUNE=--allow-tuning   # bench.py refuses PIXPATH_* overrides without it (and records them with it)
