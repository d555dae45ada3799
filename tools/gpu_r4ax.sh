# round-4: argsorts started before the upload -- fmin loop / tie order / tpe.suggest GPU tests, then the default line
set -o pipefail
O=gpurun_out/r4ax
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_fmin_loop.py tests/test_tie_order.py tests/test_tpe_gpu.py tests/test_batch.py tests/test_value_only.py tests/test_parallel.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py > $O/bench_default.log 2>&1
