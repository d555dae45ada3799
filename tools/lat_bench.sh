# the bench's tpe.suggest latency field alone (config 3, C = 24), twice
set -e
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --unscreened-steps 0 > gpurun_out/lb$i.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lb$i.log') if l.startswith('{')][-1]); print('latency', d['suggest_latency_ms'])"
done
