# SI/TI parity + A/B of the current library against tools/libvariants/*.so (bench, 2 reps).
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_siti.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_siti.log 2>&1; rc=$?
tail -2 gpurun_out/pt_siti.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt_siti.log | head -5
[ $rc -ne 0 ] && exit $rc
bash tools/ablate_lib.sh
#bash tools/gpu_counters.sh siti siti > gpurun_out/ctr_siti.txt 2>&1; tail -60 gpurun_out/ctr_siti.txt
