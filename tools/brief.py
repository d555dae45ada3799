"""Short summary of a bench log (last JSON line) and its kernel stats.
    python tools/brief.py gpurun_out/<tag>"""
import json
import os
import subprocess
import sys

d = sys.argv[1]
line = [x for x in open(os.path.join(d, 'bench.log')) if x.startswith('{')][-1]
j = json.loads(line)
print('value %.4g  ms_per_step %.3f' % (j['value'], j['ms_per_step']))
for k in ('step', 'per_family_ms', 'screened_equals_fp64'):
    print(k, json.dumps(j.get(k))[:400])
print('screen', {k: j['screen'][k] for k in ('hot_listed_fraction', 'screen_kernel_ms', 'other_dense_ms', 'rescored_per_step')})
ks = os.path.join(d, 'trace', 'run_kernel_stats.csv')
if os.path.exists(ks):
    subprocess.call([sys.executable, os.path.join(os.path.dirname(__file__), 'kstats.py'), ks])
