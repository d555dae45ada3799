# round-4: bit-word loads 4 in flight (product) against one-at-a-time (var_r4wave),
# and the product at 4 workgroups per CU (var_lb4)
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4wave.so timeout -k 10 200 python -u tools/ab_winners.py $O/wave.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/wave.npz $O/prod.npz >> $O/ab.log 2>&1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in "" tools/var_r4wave.so tools/var_lb4.so "" tools/var_r4wave.so tools/var_lb4.so; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q >> $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
