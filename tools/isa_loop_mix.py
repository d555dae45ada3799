"""Instruction mix of the innermost loop containing a marker instruction in a
hipcc --save-temps .s file (used to count VALU work per eval)."""
import collections
import re
import sys


def loop_mix(path, kernel_prefix, marker='v_rndne_f64'):
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel_prefix) and ':' in l and not l.startswith('\t'))
    end = next(i for i in range(start, len(lines)) if 's_endpgm' in lines[i])
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            labels[m.group(1)] = i
    mk = next(i for i, l in enumerate(body) if marker in l)
    # innermost backward branch that encloses the marker
    best = None
    for i, l in enumerate(body):
        m = re.search(r's_cbranch_\w+\s+(\.LBB\w+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] <= mk <= i:
            if best is None or i - labels[m.group(1)] < best[1] - best[0]:
                best = (labels[m.group(1)], i)
    mix = collections.Counter()
    for l in body[best[0]:best[1] + 1]:
        t = l.strip().split()
        if t and (t[0].startswith('v_') or t[0].startswith('ds_') or t[0].startswith('s_load')):
            mix[t[0]] += 1
    return mix


if __name__ == '__main__':
    mix = loop_mix(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
    for k, v in mix.most_common():
        print('%4d %s' % (v, k))
