#!/usr/bin/env python3
"""Compact issue sequence of a kernel in a hipcc -S listing: M mfma, f fma, x mul, G global
load, R ds_read, W ds_write, [v(n) l(n)] waits, |B| barrier.  usage: seq.py listing.s SUBSTRING"""
import re
import sys

s = open(sys.argv[1]).read()
name = [x for x in re.findall(r'^(_Z[^:\s]*):', s, re.M) if sys.argv[2] in x][0]
body = s[s.index(name + ':'):]
body = body[:body.index('.Lfunc_end')]
out = []
for l in (x.strip() for x in body.split('\n')):
    if not l:
        continue
    op = l.split()[0]
    if op.startswith('v_mfma'):
        out.append('M')
    elif 'fma' in op:
        out.append('f')
    elif op.startswith(('v_pk_mul', 'v_mul_f32')):
        out.append('x')
    elif op == 's_waitcnt':
        out.append('[' + l.split(None, 1)[1].replace('vmcnt', 'v').replace('lgkmcnt', 'l') + ']')
    elif op.startswith('global_load'):
        out.append('G')
    elif op.startswith('ds_read'):
        out.append('R')
    elif op.startswith('ds_write'):
        out.append('W')
    elif op.startswith('scratch'):
        out.append('S')
    elif op.startswith('s_barrier'):
        out.append('|B|')
    elif op.startswith('.LBB'):
        out.append('\n' + op + '\n')
print(''.join(out))
