# round-4: the order-free first build + index beside the tie orders for every
# label count (overlap-min-dense 0) vs the default (8): whole step, shards
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0"
for v in 8 0 8 0; do
  timeout -k 10 200 python -u bench.py $Q --overlap-min-dense $v >> $O/bench_o$v.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py $Q --labels 4 --no-projection --overlap-min-dense $v >> $O/bench4_o$v.log 2>&1 || exit 1
done
