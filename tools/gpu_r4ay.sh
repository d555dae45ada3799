# round-4: A/B on one box -- early argsorts before vs after the history upload (config 3 line, 3 alternations)
set -o pipefail
O=gpurun_out/r4ay
mkdir -p $O
for i in 1 2 3; do
  for e in 0 1; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-other-configs --no-agreement --no-cpu-baseline --no-latency --early-upload $e > $O/bench_e${e}_$i.log 2>&1 || exit 1
  done
done
