# round-4: order-free first build + argsorts beside it also without an index
# (tpe.suggest at 24 candidates): tests, then the suggest latency A/B
set -o pipefail
O=gpurun_out/r4an
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tpe_gpu.py tests/test_tie_order.py tests/test_fmin_loop.py tests/test_batch.py tests/test_api.py tests/test_config1.py > $O/pytest.log 2>&1 || exit 1
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --no-agreement --unscreened-steps 0 --no-projection"
for v in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py $Q --early-orders $v >> $O/bench_e$v.log 2>&1 || exit 1
done
