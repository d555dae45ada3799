# round-4: one atomic per workgroup for the waves' remainders (product),
# and k_hot_bx over 4096 / 2560 workgroups per round (variants); whole round
# and the label-shard projection
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0"
for v in "" tools/var_wgs4096.so tools/var_wgs2560.so; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q >> $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
