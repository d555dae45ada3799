# round-4: config 5 with the known labels' argsorts started before the first build (early orders) on and off
set -o pipefail
O=gpurun_out/r4ap
mkdir -p $O
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0 --no-projection"
for v in 1 0 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --config 5 $Q --early-orders $v >> $O/bench_c5_e$v.log 2>&1 || exit 1
done
