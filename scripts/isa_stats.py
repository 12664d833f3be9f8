#!/usr/bin/env python3
"""Instruction mix of one kernel in a device .s (diagnostic):  isa_stats.py FILE.s NAME_PREFIX [--print]"""
import sys
from collections import Counter

s = open(sys.argv[1]).read().split('\n')
st = [i for i, l in enumerate(s) if l.startswith(sys.argv[2]) and ':' in l][0]
b = []
for l in s[st + 1:]:
    if l.startswith('.Lfunc_end'):
        break
    t = l.strip()
    if '--print' in sys.argv and t and not t.startswith(('.', ';')):
        print(t)
    if t and not t.startswith(('.', ';')) and not t.endswith(':'):
        b.append(t)
c = Counter(l.split()[0] for l in b)
cls = Counter(('valu' if k.startswith('v_') else 'salu' if k.startswith('s_') else k.split('_')[0]) for k in (l.split()[0] for l in b))
print(s[st].split(':')[0][:80], 'static instructions:', len(b), dict(cls))
print(sorted(c.items(), key=lambda x: -x[1])[:40])
