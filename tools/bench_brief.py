"""One line per bench log: workload, ms/step, value, roofline frac and the
screen's split (tools for reading gpurun_out/ logs).

    python tools/bench_brief.py gpurun_out/a.log [more.log ...]
"""
import json
import sys


def brief(path):
    for line in open(path):
        if line.startswith('{"metric"'):
            d = json.loads(line)
            s = d.get('screen', {})
            return ('%-10s %8.2f ms  %.3g evals/s  frac %s  screen %s ms  other %s ms  '
                    'terms %.4f  rescored %.5f' % (
                        d['config']['workload'][:10], d['ms_per_step'], d['value'],
                        d['roofline']['frac'], s.get('screen_kernel_ms'), s.get('other_dense_ms'),
                        s.get('screen_terms_fraction', 0), s.get('rescored_fraction', 0)))
    return '%s: no bench line' % path


if __name__ == '__main__':
    for p in sys.argv[1:]:
        try:
            print(brief(p))
        except OSError as e:
            print(e)
