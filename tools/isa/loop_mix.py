#!/usr/bin/env python3
"""Instruction mix of a kernel's loops in a hipcc -S listing (ISA inspection aid).

usage: loop_mix.py listing.s SUBSTRING   -- every kernel whose symbol contains SUBSTRING:
vgpr/spill counts, then per backward branch (a loop) the instruction counts of its body."""
import re
import sys
from collections import Counter


def main():
    s = open(sys.argv[1]).read()
    for name in re.findall(r'^(_Z[^:\s]*):', s, re.M):
        if sys.argv[2] not in name:
            continue
        body = s[s.index(name + ':'):]
        body = body[:body.index('.Lfunc_end')]
        meta = s[s.index('.name:           ' + name) - 2000:s.index('.name:           ' + name) + 600] \
            if ('.name:           ' + name) in s else ''
        vg = re.findall(r'\.vgpr_count:\s*(\d+)', meta)
        sp = re.findall(r'\.vgpr_spill_count:\s*(\d+)', meta)
        print(name, 'vgpr', vg[-1:] , 'spill', sp[-1:])
        lines = [l.strip() for l in body.split('\n')]
        labels = {}
        for i, l in enumerate(lines):
            m = re.match(r'^(\.LBB[\w_]+):', l)
            if m:
                labels[m.group(1)] = i
        for i, l in enumerate(lines):
            m = re.match(r'^s_cbranch_\w+\s+(\.LBB[\w_]+)', l) or re.match(r'^s_branch\s+(\.LBB[\w_]+)', l)
            if m and m.group(1) in labels and labels[m.group(1)] < i:
                seg = [x for x in lines[labels[m.group(1)]:i + 1] if x and not x.startswith(('.', ';'))]
                c = Counter(x.split()[0] for x in seg)
                print('  loop %s: %d instr' % (m.group(1), len(seg)), dict(c.most_common(24)))


if __name__ == '__main__':
    main()
