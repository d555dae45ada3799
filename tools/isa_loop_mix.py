"""Instruction mix of the innermost loop of a kernel that contains a marker
instruction at least `min_count` times, from a hipcc --save-temps .s file
(used to count VALU work per (candidate, component) eval).

    python tools/isa_loop_mix.py <file.s> <kernel symbol prefix> [marker] [min_count]
"""
import collections
import re
import sys


def loop_mix(path, kernel_prefix, marker='v_ldexp_f64', min_count=4):
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel_prefix) and l.rstrip().endswith(':')
                 or (l.startswith(kernel_prefix) and ': ;' in l))
    end = next(i for i in range(start, len(lines)) if 's_endpgm' in lines[i])
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.search(r's_cbranch_\w+\s+(\.LBB\w+)', l) or re.search(r's_branch\s+(\.LBB\w+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            lo = labels[m.group(1)]
            if sum(marker in b for b in body[lo:i + 1]) >= min_count:
                if best is None or i - lo < best[1] - best[0]:
                    best = (lo, i)
    mix = collections.Counter()
    for l in body[best[0]:best[1] + 1]:
        t = l.strip().split()
        if t and (t[0].startswith('v_') or t[0].startswith('ds_') or t[0].startswith('s_')):
            mix[t[0]] += 1
    return mix


if __name__ == '__main__':
    mix = loop_mix(sys.argv[1], sys.argv[2], *(sys.argv[3:4] or ['v_ldexp_f64']),
                   *([int(sys.argv[4])] if len(sys.argv) > 4 else []))
    valu = sum(v for k, v in mix.items() if k.startswith('v_'))
    per = mix.get('v_ldexp_f64', 1)
    print('VALU instructions in loop: %d (%.2f per v_ldexp_f64 = per eval)' % (valu, valu / per))
    for k, v in mix.most_common():
        print('%5d %s' % (v, k))
