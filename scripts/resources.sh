#!/bin/bash
# Per-kernel VGPR / scratch / occupancy of one translation unit (compile only).
# usage: resources.sh tu_shade.hip [-DPT_FT=16] [kernel-substring]
D=$(dirname "$0")/../pbrt-v3-light-portals_amd
TU=$1; shift
DEF=""; [ $# -gt 0 ] && [[ "$1" == -D* ]] && { DEF=$1; shift; }
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-approx-transcendentals $EXTRA $DEF -I"$D/../include" \
  --cuda-device-only -c -o /tmp/ptres.o "$D/csrc/$TU" -Rpass-analysis=kernel-resource-usage 2>&1 | \
python3 -c '
import re, sys
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m: cur = m.group(1); info = {}; continue
    for k in ("VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]"):
        m = re.search(re.escape(k) + r": (\d+)", l)
        if m and cur: info[k.split()[0]] = m.group(1)
    if cur and "Occupancy" in l:
        if pat in cur: print("%-70s vgpr=%s scratch=%s waves=%s" % (cur[:70], info.get("VGPRs"), info.get("ScratchSize"), info.get("Occupancy")))
        cur = None
' "${1:-}"
