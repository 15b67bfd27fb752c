# SQ / TCC counters of the FFV1 kernels (bench --workload ffv1, one encode and
# one decode of 600 frames per pass), plus FETCH_SIZE / WRITE_SIZE passes.
# Usage: bash tools/gpu_ffv1_pmc_r5.sh TAG
set -o pipefail
TAG=$1
D=gpurun_out/fctr_$TAG
mkdir -p $D
export TMPDIR=/tmp
RUN="python3 bench.py --workload ffv1 --steps 1 --warmup 0 --no-cpu-baseline --ffv1-concurrent 1"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" \
           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o run -- $RUN > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $D/p$i.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- $RUN > $D/kt.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/summarize_counters.py $D > $D/summary.txt
cat $D/summary.txt
grep -E "ffv1" $D/kt/run_kernel_stats.csv | cut -d, -f1-4
