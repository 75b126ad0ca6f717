"""Instruction mix of the hottest loop of each kernel in a gfx950 .s file (dev diagnostics).

usage: python tools/loop_stats.py file.s substring [substring ...]
"""
import re
import sys


def loop_stats(s, name):
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    lines = [l.strip() for l in s[i:j].split('\n')]
    labels = {}
    for k, l in enumerate(lines):
        m = re.match(r'^(\.LBB\d+_\d+):', l)
        if m:
            labels[m.group(1)] = k
    best = None
    for k, l in enumerate(lines):
        m = re.match(r's_(?:cbranch_\w+|branch) (\.LBB\d+_\d+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            seg = lines[labels[m.group(1)]:k + 1]
            nm = sum(x.startswith('v_mfma') for x in seg)
            if nm and (best is None or nm > best[0]):
                best = (nm, seg)
    if best is None:
        return None
    nm, seg = best
    cnt = lambda f: sum(1 for x in seg if f(x))
    return dict(mfma=nm,
                valu=cnt(lambda x: x.startswith('v_') and not x.startswith('v_mfma')),
                salu=cnt(lambda x: x.startswith('s_') and not x.startswith(('s_waitcnt', 's_nop'))),
                vmem=cnt(lambda x: x.startswith(('buffer_', 'global_'))),
                lds=cnt(lambda x: x.startswith('ds_')),
                waitcnt=cnt(lambda x: x.startswith('s_waitcnt')))


if __name__ == '__main__':
    s = open(sys.argv[1]).read()
    names = re.findall(r'^(_Z\w+):', s, re.M)
    for sub in sys.argv[2:]:
        for n in names:
            if sub in n:
                print(n[:110], loop_stats(s, n))
