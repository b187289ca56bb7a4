#!/bin/bash
# Kernel resource usage (VGPRs, scratch, occupancy) of the default render kernels for depth <= RT_MAX_B
# (default 3: the c1/c2/c3/c5 kernels), device-only compile.  Extra hipcc flags as arguments, e.g.
#   bash tools/resusage.sh -DRT_MINW_CULL=4
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/ray_tracer_fragment_shader_amd/csrc
out=$(mktemp -d)
( cd "$SRC" && for b in $(seq 0 ${RT_MAX_B:-3}); do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-function \
    --offload-arch=gfx950 --cuda-device-only -S "$@" rt_render_b$b.hip -o "$out/k$b.s" \
    -Rpass-analysis=kernel-resource-usage 2> "$out/ru$b.txt" & done; wait; cat "$out"/ru*.txt > "$out/ru.txt" )
python3 - "$out/ru.txt" <<'EOF'
import re, sys
cur = None
rows = {}
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for name, r in rows.items():
    m = re.search(r"rt_render_kernelILi(\d)ELi(\d)ELi(\d)ELb(\d)ELb(\d)ELi(\d+)E", name)
    if not m:
        continue
    B, LDS, MINW, TR, CULL, WG = m.groups()
    if LDS != "0" or WG != "64":
        continue
    print(f"B={B} MINW={MINW} TRANSP={TR} CULL={CULL}: VGPR {r.get('VGPRs')} scratch {r.get('ScratchSize [bytes/lane]')} "
          f"vspill {r.get('VGPRs Spill')} sspill {r.get('SGPRs Spill')} occ {r.get('Occupancy [waves/SIMD]')}")
EOF
rm -rf "$out"
