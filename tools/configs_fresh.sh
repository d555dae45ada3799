#!/bin/bash
# fresh-posterior bench lines of configs 2, 4 and 5 (config 3 is the default line)
set -u
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in 2 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-latency --no-cpu-baseline > $OUT/c$c.log 2>&1 || { tail -20 $OUT/c$c.log; exit 1; }
  python - $OUT/c$c.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]
d = json.loads(l)
print(sys.argv[1], 'ms_per_step %.3f' % d['ms_per_step'], 'value %.3g' % d['value'], json.dumps(d.get('step'))[:300], d.get('screened_equals_fp64'))
PY
done
