# round-4: armed prepare (the build queues the index) -- whole GPU suite, bench, traced short bench
set -o pipefail
O=gpurun_out/r4av
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-other-configs --no-agreement --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-other-configs --no-agreement --no-cpu-baseline --no-latency > $O/bench_trace.log 2>&1
