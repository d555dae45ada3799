# round-4 check: the new parity / no-sync / value-only tests, then the bench
set -o pipefail
mkdir -p gpurun_out/r4a
export NEAR_TIE_OUT=gpurun_out/r4a
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_value_only.py tests/test_parallel.py tests/test_screen.py tests/test_tie_order.py tests/test_batch.py > gpurun_out/r4a/pytest_a.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_near_tie_agreement.py > gpurun_out/r4a/pytest_nt.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r4a/bench.log 2>&1
