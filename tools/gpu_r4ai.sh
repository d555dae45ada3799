# round-4: the rebuild's orders from pinned memory vs pageable, configs 3 and 5; the fmin-loop tests
set -o pipefail
O=gpurun_out/r4ai
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fmin_loop.py tests/test_tie_order.py tests/test_tpe_gpu.py > $O/pytest.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0 --no-projection"
for v in 1 0 1 0; do
  for c in 3 5; do
    timeout -k 10 200 python -u bench.py --config $c $Q --pin-orders $v >> $O/bench_c${c}_p$v.log 2>&1 || exit 1
  done
done
