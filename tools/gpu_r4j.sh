# round-4: periodic hot-buffer flush (product) against HEAD before it (var_r4pre):
# winners identical, bracket time; plus the commits around the slowdown
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4pre.so timeout -k 10 200 python -u tools/ab_winners.py $O/pre.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/pre.npz $O/prod.npz >> $O/ab.log 2>&1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in "" tools/var_r4pre.so tools/var_r3end.so tools/var_r4a2.so tools/var_r4base.so; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q > $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
