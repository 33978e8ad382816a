#!/usr/bin/env python3
"""Attribute one kernel's device instructions to source functions, from a
-gline-tables-only assembly listing (.loc directives; inlined code counts
toward the innermost function).  usage: isa_attrib.py listing.s kernel-prefix"""
import bisect
import collections
import os
import re
import sys

s = open(sys.argv[1]).read()
files = {m.group(1): m.group(3) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', s, re.M)}
a = s.index('\n' + sys.argv[2])
a = s.index(':', a)
e = s.index('s_endpgm', a)
cur = ('?', 0)
cnt = collections.Counter()
for l in s[a:e].split('\n'):
    t = l.strip()
    if t.startswith('.loc'):
        p = t.split()
        cur = (os.path.basename(files.get(p[1], p[1])), int(p[2]))
        continue
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    cnt[cur] += 1
csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pbrt-v3-light-portals_amd', 'csrc')
fm = {}
for f in os.listdir(csrc):
    starts = []
    for i, l in enumerate(open(os.path.join(csrc, f), errors='replace').read().split('\n'), 1):
        m = re.match(r'^(?:__device__|__global__|PTHD|static|inline|template)[^(]*?(\w+)\(', l)
        if m:
            starts.append((i, m.group(1)))
    fm[f] = starts
agg = collections.Counter()
for (f, ln), c in cnt.items():
    st = fm.get(f)
    if not st:
        agg[(f, '?')] += c
        continue
    i = bisect.bisect_right([x[0] for x in st], ln) - 1
    agg[(f, st[i][1] if i >= 0 else '?')] += c
print('total', sum(agg.values()))
for k, v in agg.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{v:7d}  {k[0]}:{k[1]}")
