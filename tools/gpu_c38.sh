# Config-3 strip_kernel study: variant A/B (product / staging swap / H-read
# rotation) on config3-8, config3-10 and config2, the ablation bits of the
# measurement build on config3-8, and the LDS counters of config3-8.
# usage: bash tools/gpu_c38.sh TAG
set -o pipefail
TAG=${1:-c38}
export TMPDIR=/tmp
O=gpurun_out/c38_$TAG; mkdir -p $O
ARGS="--allow-tuning --steps 10 --warmup 3 --pvs-total 32 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e"
show() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', r['avg_launch_ms'], r['frac'])"; }
for rep in 1 2; do
for wl in config3-8 config3-10 config2; do
for v in product swap rot; do
  if [ $v = product ]; then lib=$PWD/processing-chain_amd/pixpath/libpixpath.so; else lib=$PWD/tools/ablate/libpixpath_$v.so; fi
  PIXPATH_LIB=$lib timeout -k 10 120 python3 bench.py $ARGS --workload $wl > $O/$wl-$v.json 2> $O/$wl-$v.err || { tail -3 $O/$wl-$v.err; exit 1; }
  show $O/$wl-$v.json "$wl $v"
done
done
done
for dbg in 0 1 2 4 6 8; do
  PIXPATH_LIB=$PWD/tools/ablate/libpixpath_ablate.so PIXPATH_SCALE_DEBUG=$dbg timeout -k 10 120 python3 bench.py $ARGS --workload config3-8 > $O/abl$dbg.json 2> $O/abl$dbg.err || { tail -3 $O/abl$dbg.err; exit 1; }
  show $O/abl$dbg.json "config3-8 debug $dbg"
done
PK="--allow-tuning --steps 1 --warmup 0 --pvs-total 2 --pool 2 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e --workload config3-8"
for v in product swap; do
  if [ $v = product ]; then lib=$PWD/processing-chain_amd/pixpath/libpixpath.so; else lib=$PWD/tools/ablate/libpixpath_$v.so; fi
  i=0; mkdir -p $O/ctr_$v
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    PIXPATH_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/ctr_$v/p$i -o run -- python3 bench.py $PK > $O/ctr_$v/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/ctr_$v/p$i.log; exit 1; }
  done
  echo "### counters $v"; python3 tools/summarize_counters.py $O/ctr_$v | grep -A20 "strip_kernel"
done
