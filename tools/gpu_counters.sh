# SQ/TCP counter passes on the isolated kernels.  Usage: bash tools/gpu_counters.sh TAG [which]
set -o pipefail
TAG=${1:-c}; WHICH=${2:-both}
mkdir -p gpurun_out/ctr_$TAG
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" \
           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/ctr_$TAG/p$i -o run -- python3 tools/prof_kernels.py --which $WHICH $PK_ARGS > gpurun_out/ctr_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ctr_$TAG/kt -o run -- python3 tools/prof_kernels.py --which $WHICH $PK_ARGS > gpurun_out/ctr_$TAG/kt.log 2>&1
python3 tools/summarize_counters.py gpurun_out/ctr_$TAG
