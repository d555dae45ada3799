# round-4: config 4 projected over 8 label shards (1-2 labels each) vs candidate shards
set -o pipefail
O=gpurun_out/r4am
mkdir -p $O
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0"
for s in labels auto labels auto; do
  timeout -k 10 200 python -u bench.py --config 4 $Q --shard $s >> $O/bench_c4_$s.log 2>&1 || exit 1
done
