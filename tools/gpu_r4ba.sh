# round-4: quantized + categorical labels on the aux stream -- whole GPU suite, then A/B on one box
set -o pipefail
O=gpurun_out/r4ba
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  for c in 0 1; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-other-configs --no-agreement --no-cpu-baseline --no-latency --aux-families $c > $O/bench_a${c}_$i.log 2>&1 || exit 1
  done
done
for c in 0 1; do
  timeout -k 10 300 python -u bench.py --config 5 --steps 6 --warmup 2 --no-agreement --no-cpu-baseline --no-latency --aux-families $c > $O/bench5_a${c}.log 2>&1 || exit 1
done
