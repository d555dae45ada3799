# round-4: which commit slowed k_hot_bx (bench bracket of k_hot_bx + k_screen_hot)
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in tools/var_r3end.so tools/var_r4a1.so tools/var_r4a2.so tools/var_r4base.so ""; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q > $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
