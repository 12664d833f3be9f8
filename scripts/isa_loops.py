#!/usr/bin/env python3
"""Per-loop instruction mix of one kernel in a device .s (diagnostic):  isa_loops.py FILE.s NAME_PREFIX"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read().split('\n')
st = [i for i, l in enumerate(s) if l.startswith(sys.argv[2]) and ':' in l][0]
en = st
while not s[en].startswith('.Lfunc_end'):
    en += 1
body = s[st:en]
labels = {l.split(':')[0]: i for i, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)}
for i, l in enumerate(body):
    m = re.search(r's_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)', l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < i:
            seg = [x.strip() for x in body[labels[t]:i + 1] if x.strip() and not x.strip().startswith(('.', ';'))]
            c = Counter(x.split()[0] for x in seg)
            v = sum(n for k, n in c.items() if k.startswith('v_') and 'mfma' not in k)
            mf = sum(n for k, n in c.items() if 'mfma' in k)
            print('loop', t, 'len', len(seg), 'mfma', mf, 'valu', v)
            print(' ', sorted(c.items(), key=lambda x: -x[1])[:24])
