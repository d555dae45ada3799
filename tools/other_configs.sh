# bench lines of configs 2, 4, 5 (short) and a kernel-trace summary of config 5
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--no-cpu-baseline --no-latency --unscreened-steps 0"
for c in 2 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 $Q > gpurun_out/c$c.log 2>&1
  echo "config $c: $(python tools/bench_brief.py gpurun_out/c$c.log) $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c$c.log') if l.startswith('{')][-1]); print(d['per_family_ms'], d.get('screen',{}).get('hot_listed_fraction'))")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run --output-format csv -- python -u bench.py --config 5 --steps 3 --warmup 1 $Q > gpurun_out/c5prof.log 2>&1
echo traced
