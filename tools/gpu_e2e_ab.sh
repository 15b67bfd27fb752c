# e2e_avpvs: shared encode stream (serial encodes) vs private streams, twice each.
set -o pipefail
for rep in 1 2; do
EXTRA="--e2e-encode shared" bash tools/gpu_e2e.sh e2e_shared_$rep || exit 1
EXTRA="--e2e-encode private" bash tools/gpu_e2e.sh e2e_private_$rep || exit 1
done
