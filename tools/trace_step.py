"""Timeline of one fmin step from a rocprofv3 --kernel-trace --hip-runtime-trace
[--memory-copy-trace] csv directory: host API calls (H), kernels (K) and
copies (M) in start order, from the k-th last launch of a marker kernel (the
step's first kernel) to the next one, with the host-side gaps between API
calls and the device idle time between kernels -- where a step's fixed
latency goes.

    python tools/trace_step.py <trace dir> [marker=k_split] [k=2] [min_us=0]
"""
import csv
import glob
import sys


def load(d):
    ev = []
    for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K', r['Kernel_Name'][:80],
                       r.get('Correlation_Id')))
    for f in glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'M', r.get('Direction', ''),
                       r.get('Correlation_Id')))
    for f in glob.glob(d + '/**/*hip_api_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'H', r['Function'],
                       r.get('Correlation_Id')))
    ev.sort()
    return ev


def main(d, marker='k_split', k=2, min_us=0.0):
    ev = load(d)
    starts = [i for i, e in enumerate(ev) if e[2] == 'K' and marker in e[3]]
    a = starts[-int(k)]
    b = starts[-int(k) + 1] if int(k) > 1 else len(ev)
    seg = ev[a:b]
    # include the host calls that launched the first kernels (start before it)
    t0 = seg[0][0]
    hosts = [e for e in ev[:a] if e[2] == 'H' and e[1] >= t0 - 2000000]
    t0 = min([t0] + [e[0] for e in hosts[-40:]])
    last_dev_end = None
    dev_busy = 0
    for e in sorted(hosts[-40:] + seg):
        dur = (e[1] - e[0]) / 1e3
        if e[2] in 'KM':
            gap = (e[0] - last_dev_end) / 1e3 if last_dev_end else 0.0
            last_dev_end = max(last_dev_end or 0, e[1])
            dev_busy += e[1] - e[0]
            tag = 'dev gap %7.1f' % gap
        else:
            tag = ' ' * 15
        if dur >= float(min_us) or e[2] == 'K':
            print('%9.1f us  %s %s dur %8.1f  %s' % ((e[0] - t0) / 1e3, e[2], tag, dur, e[3]))
    span = (seg[-1][1] - seg[0][0]) / 1e3
    print('step span %.1f us, device busy %.1f us (kernels + copies)' % (span, dev_busy / 1e3))


if __name__ == '__main__':
    main(*sys.argv[1:])
