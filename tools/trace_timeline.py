"""Print the kernel / copy timeline from the k-th last launch of a marker
kernel on (k = 1: the last), from a rocprofv3 --kernel-trace
[--memory-copy-trace] [--hip-trace] csv directory.

    python tools/trace_timeline.py <trace dir> [marker=k_split] [k=1] [before=3] [count=40]
"""
import csv
import glob
import sys


def main(d, marker='k_split', k=1, before=3, count=40):
    ev = []
    for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K ' + r['Kernel_Name'][:70]))
    for f in glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                       'M %s %s' % (r.get('Direction', ''), r.get('Size', ''))))
    for f in glob.glob(d + '/**/*hip_api_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'A ' + r['Function'][:60]))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if marker in e[2]]
    s = max(idx[-int(k)] - int(before), 0)
    t0 = prev = ev[s][0]
    for e in ev[s:s + int(count)]:
        print('%8.1f us  dur %6.1f  gap %6.1f  %s' % ((e[0] - t0) / 1e3, (e[1] - e[0]) / 1e3,
                                                    (e[0] - prev) / 1e3, e[2]))
        prev = e[1]


if __name__ == '__main__':
    main(*sys.argv[1:])
