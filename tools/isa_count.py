#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing (tools only).
   python tools/isa_count.py rsock_amd/rsk_kernels.s k_tag_table [--from LINE --to LINE]"""
import collections
import re
import sys


def body(lines, pat):
    for i, l in enumerate(lines):
        m = re.match(r'^(_Z\S+):\s*;', l)
        if m and pat in m.group(1):
            out = []
            for x in lines[i + 1:]:
                if x.startswith('.Lfunc_end'):
                    break
                out.append(x)
            yield m.group(1), out


def main():
    lines = open(sys.argv[1]).read().split('\n')
    for name, b in body(lines, sys.argv[2]):
        ins = [l.strip().split()[0] for l in b if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        salu = sum(v for k, v in c.items() if k.startswith('s_'))
        print(name[:90], 'total', len(ins), 'v_', valu, 's_', salu)
        print('  ', sorted(c.items(), key=lambda x: -x[1])[:24])


if __name__ == '__main__':
    main()
