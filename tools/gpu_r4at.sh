# round-4: register-cached k_split -- build/tie-order parity, then a short profiled bench
set -o pipefail
O=gpurun_out/r4at
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_build.py tests/test_tie_order.py tests/test_fmin_loop.py tests/test_posterior.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 -u bench.py --steps 8 --warmup 3 --no-other-configs --no-agreement --no-cpu-baseline > $O/bench.log 2>&1
