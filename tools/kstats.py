"""Per-kernel table (per launch ms, share) of a rocprofv3 --stats csv:

    python tools/kstats.py gpurun_out/<dir>/run_kernel_stats.csv [top]
"""
import csv
import re
import sys


def main(path, top=16):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    for r in rows[:top]:
        n = re.sub(r'\(anonymous namespace\)::|void |rocprim::ROCPRIM_\d+_NS::detail::', '', r['Name'])
        print('%-64s %5s calls %8.3f ms/launch %5.1f%%' % (
            n[:64], r['Calls'], float(r['AverageNs']) / 1e6, 100 * float(r['TotalDurationNs']) / tot))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 16)
