# k_hot_bx sweep: slots per thread (TPE_HOT_R) x workgroups per round (TPE_HOT_WGS)
set -e
for cfg in "8 16384" "8 32768"; do
  set -- $cfg
  TPE_HOT_R=$1 TPE_HOT_WGS=$2 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-latency --unscreened-steps 0 > gpurun_out/hr$1_$2.log 2>&1
  echo "R=$1 WGS=$2 $(python tools/bench_brief.py gpurun_out/hr$1_$2.log) $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/hr$1_$2.log') if l.startswith('{')][-1]); print(d['per_family_ms'])")"
done
