#!/usr/bin/env python3
"""Instruction classes per loop body (back-edge to an earlier label) of one
kernel in a device assembly listing — a static view of where a kernel's VALU
issue goes (see tools/asm_stats.py for how to produce the listing).

  python tools/loop_stats.py build/k.s <kernel-symbol-substring>
"""
import re
import sys
from collections import Counter

TRANS = ('v_sin', 'v_cos', 'v_rcp', 'v_sqrt', 'v_rsq', 'v_exp', 'v_log')


def classify(op):
    if op.startswith('v_pk_'):
        return 'v_pk'
    if op.startswith(TRANS):
        return 'trans'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('global_load'):
        return 'gload'
    if op.startswith('global_store'):
        return 'gstore'
    if op.startswith('s_waitcnt'):
        return 'wait'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main(path, sub):
    s = open(path).read()
    m = re.search(r'^(_Z\S*' + re.escape(sub) + r'\S*):', s, re.M)
    i = m.start()
    j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    labels = {}
    for k, line in enumerate(body):
        mm = re.match(r'^(\.LBB\S+):', line)
        if mm:
            labels[mm.group(1)] = k
    print(m.group(1)[:100])
    for k, line in enumerate(body):
        mm = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\S+)', line)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < k:
            a = labels[mm.group(1)]
            ops = [x.split()[0] for x in body[a:k + 1] if x.startswith('\t') and not x.startswith(('\t;', '\t.'))]
            c = Counter(classify(o) for o in ops)
            print(f"  loop {mm.group(1)} lines {a}-{k}: {len(ops)} instr {dict(c)}")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
