set -e
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-latency --unscreened-steps 0 > gpurun_out/q.log 2>&1
echo "$(python tools/bench_brief.py gpurun_out/q.log) $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/q.log') if l.startswith('{')][-1]); print(d['per_family_ms'])")"
