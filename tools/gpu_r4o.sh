# round-4: coarse LDS map of the nonzero bit words (product) against every
# candidate loading its word (var_r4hoist); winners, bracket, kernel trace
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4hoist.so timeout -k 10 200 python -u tools/ab_winners.py $O/hoist.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/hoist.npz $O/prod.npz >> $O/ab.log 2>&1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in "" tools/var_r4hoist.so "" tools/var_r4hoist.so; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q >> $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_screen.py tests/test_fmin_loop.py > $O/pytest.log 2>&1
