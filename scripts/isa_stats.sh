#!/bin/bash
# Per-kernel code size and scratch use of one translation unit (device ISA):
# instruction lines, scratch ops that are register spills/reloads and the
# rest (private arrays).  usage: isa_stats.sh tu_hero.hip [kernel-substring]
set -e
D=$(dirname "$0")/../pbrt-v3-light-portals_amd
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-approx-transcendentals $EXTRA -I"$D/../include" \
  --cuda-device-only -S -o /tmp/isa/out.s "$D/csrc/$1" 2>/dev/null
python3 - "${2:-k_}" <<'P'
import re, sys
s = open('/tmp/isa/out.s').read()
for m in re.finditer(r'^(_ZN2pt\w+):', s, re.M):
    name = m.group(1)
    if sys.argv[1] not in name: continue
    e = s.index('s_endpgm', m.end())
    lines = [l for l in s[m.end():e].split('\n') if l.strip() and not l.strip().startswith(('.', ';')) and not l.strip().endswith(':')]
    sc = [l for l in lines if 'scratch_' in l]
    sp = [l for l in sc if 'Spill' in l or 'Reload' in l]
    print(f"{name[:60]:60s} instrs={len(lines):6d} scratch_ops={len(sc):5d} spill={len(sp):5d}")
P
