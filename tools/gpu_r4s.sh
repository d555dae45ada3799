# round-4: k_hot_bx workgroups per cell with a floor of 6 tiles each
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0"
timeout -k 10 200 python -u bench.py $Q > $O/bench_c3.log 2>&1 || exit 1
for c in 2 4 5; do timeout -k 10 200 python -u bench.py --config $c $Q > $O/bench_c$c.log 2>&1 || exit 1; done
