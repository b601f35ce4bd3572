#!/usr/bin/env python3
"""Runs of >= N consecutive v_mov in a kernel's ISA (register shuffles where
code paths join), with their block and loop depth.
  tools/isa_movruns.py <file.s> <kernel-substring> [N]"""
import re
import sys

s = open(sys.argv[1]).read()
pat, N = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8
parts = re.split(r'\n(_Z[\w]+):\s*(?:;[^\n]*)?\n', s)
for name, body in zip(parts[1::2], parts[2::2]):
    if pat not in name:
        continue
    lines = body.split('.Lfunc_end')[0].split('\n')
    hdr, depth, run, start = '', 0, 0, 0
    for i, l in enumerate(lines + ['']):
        if re.match(r'^(\.LBB\S+:|; %bb\.\d+:)', l):
            hdr = l.split(':')[0]
            m = re.search(r'Depth=(\d+)', l)
            depth = int(m.group(1)) if m else 0
        t = l.strip()
        if t.startswith('v_mov_b32') or t.startswith('v_mov_b64'):
            if run == 0:
                start, bh, bd = i, hdr, depth
            run += 1
        elif t and not t.startswith(';') and not t.startswith('s_nop'):
            if run >= N:
                print(f"{name[:50]} line {start} {bh} depth {bd}: {run} movs")
            run = 0
