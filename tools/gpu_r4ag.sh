# round-4: zero windows only for a non-empty packed re-score plan: packed-map tests, config-5 bench
set -o pipefail
O=gpurun_out/r4ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_value_only.py tests/test_screen.py tests/test_gpu_fullsize.py tests/test_batch.py tests/test_mode_mask.py > $O/pytest.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --no-projection"
timeout -k 10 200 python -u bench.py --config 5 $Q > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config 5 $Q --value-only 0 > $O/bench_c5_exact.log 2>&1
