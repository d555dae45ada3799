# round-4: deferred quantized round (TPE_OPT_MODE_MASK) tests, device merge, bench
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_fmin_loop.py tests/test_parallel.py tests/test_value_only.py tests/test_tpe_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1
