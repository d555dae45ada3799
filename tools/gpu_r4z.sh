# round-4: the aux stream at high priority (product) vs default priority (var_r4pre4)
set -o pipefail
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fmin_loop.py tests/test_tie_order.py > $O/pytest.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0"
for v in "" tools/var_r4pre4.so "" tools/var_r4pre4.so; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q >> $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
