# round-4: second-stream families off by default -- whole GPU suite, smoke, default line
set -o pipefail
O=gpurun_out/r4bb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for c in 0 1; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-other-configs --no-agreement --no-cpu-baseline --no-latency --aux-families $c > $O/bench_a${c}.log 2>&1 || exit 1
done
