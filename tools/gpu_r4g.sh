# round-4: A/B of the deferred quantized round (argsorts under the dense round)
# and of the argsort pool's size, configs 3 and 5
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for cfg in 3 5; do
  for v in "0 16" "1 16" "1 4" "0 4" "1 1"; do
    set -- $v
    timeout -k 10 200 python -u bench.py --config $cfg $Q --defer $1 --sort-threads $2 > $O/c${cfg}_d$1_t$2.log 2>&1 || exit 1
  done
done
