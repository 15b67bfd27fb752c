# Register report of every strip_kernel instance (device asm of strip_u16.hip / strip_u8.hip).
# Usage: bash tools/check_spills.sh [-a]   (prints instances with spills, or all with -a)
set -e
cd "$(dirname "$0")/../processing-chain_amd"
for f in strip_u16 strip_u8; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -x hip csrc/$f.hip --cuda-device-only -S -o /tmp/$f.s 2>/dev/null &
done
wait
python3 - "$@" <<'PY'
import re, sys
bad = 0
for f in ['/tmp/strip_u16.s', '/tmp/strip_u8.s']:
    txt = open(f).read()
    for b in txt.split('  - .agpr_count:')[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        m = re.search(r"strip_kernelI(\w)Li(\d+)ELi(\d+)ELi(\d+)E", name)
        if not m:
            continue
        vg = int(re.search(r"\.vgpr_count:\s+(\d+)", b).group(1))
        sg = int(re.search(r"\.sgpr_count:\s+(\d+)", b).group(1))
        vs = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", b).group(1))
        ss = int(re.search(r"\.sgpr_spill_count:\s+(\d+)", b).group(1))
        st = {'t': 'u16', 'h': 'u8'}[m.group(1)]
        if vs or ss or '-a' in sys.argv:
            print("%s OUTB=%s HW=%s VTM=%s  vgpr=%d sgpr=%d vspill=%d sspill=%d" % (st, m.group(2), m.group(3), m.group(4), vg, sg, vs, ss))
        bad += (vs > 0)
print("instances with VGPR spills:", bad)
PY
