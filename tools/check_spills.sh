# Register report of every strip_kernel instance (device asm of the strip_u16*/strip_u8* units).
# Usage: bash tools/check_spills.sh [-a]   (prints instances with spills, or all with -a)
set -e
cd "$(dirname "$0")/../processing-chain_amd"
for f in strip_u16 strip_u16_chain strip_u8 strip_u8_chain strip_u16_fused strip_u8_fused; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -x hip csrc/$f.hip --cuda-device-only -S -o /tmp/$f.s 2>/dev/null &
done
wait
python3 - "$@" <<'PY'
import re, sys
bad = 0
for f in ["/tmp/strip_u16.s", "/tmp/strip_u16_chain.s", "/tmp/strip_u8.s", "/tmp/strip_u8_chain.s", "/tmp/strip_u16_fused.s", "/tmp/strip_u8_fused.s"]:
    txt = open(f).read()
    for b in txt.split('  - .agpr_count:')[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        m = re.search(r"strip_kernelI(\w)Li(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", name)
        if not m:
            continue
        vg = int(re.search(r"\.vgpr_count:\s+(\d+)", b).group(1))
        sg = int(re.search(r"\.sgpr_count:\s+(\d+)", b).group(1))
        vs = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", b).group(1))
        ss = int(re.search(r"\.sgpr_spill_count:\s+(\d+)", b).group(1))
        st = {'t': 'u16', 'h': 'u8'}[m.group(1)]
        if vs or ss or '-a' in sys.argv:
            print("%s OUTB=%s HW=%s VTM=%s FUSE=%s  vgpr=%d sgpr=%d vspill=%d sspill=%d" % (st, m.group(2), m.group(3), m.group(4), m.group(5), vg, sg, vs, ss))
        bad += (vs > 0)
print("instances with VGPR spills:", bad)
PY
# every kernel of every HIP source: no private (scratch) segment
for f in scale cpvs pack siti; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -x hip csrc/$f.hip --cuda-device-only -S -o /tmp/$f.s 2>/dev/null &
done
wait
python3 - <<'PY'
import re
bad = []
for f in ["scale", "cpvs", "pack", "siti", "strip_u16", "strip_u16_chain", "strip_u8", "strip_u8_chain", "strip_u16_fused", "strip_u8_fused"]:
    txt = open('/tmp/%s.s' % f).read()
    for b in txt.split('  - .agpr_count:')[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        ps = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", b).group(1))
        if ps:
            bad.append((f, name, ps))
for x in bad:
    print("scratch: %s %s %d B" % x)
print("kernels with a private segment:", len(bad))
PY
# v_ashr_pk_u8_i32 keeps its destination's high half: a kernel that ORs more bytes
# into such a result is wrong (cpvs.hip hit this); flag every occurrence
if grep -l "v_ashr_pk_u8_i32" /tmp/scale.s /tmp/cpvs.s /tmp/pack.s /tmp/siti.s /tmp/strip_u16.s /tmp/strip_u16_chain.s /tmp/strip_u8.s /tmp/strip_u8_chain.s /tmp/strip_u16_fused.s /tmp/strip_u8_fused.s; then
  echo "v_ashr_pk_u8_i32 present: check its uses"; exit 1
fi
echo "no v_ashr_pk_u8_i32"
