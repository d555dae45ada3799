# round-4: quantized tables from the above mixtures' runs (k_qcompress): the whole GPU suite, then configs 5 and 3
set -o pipefail
O=gpurun_out/r4aq
mkdir -p $O/nt
NEAR_TIE_OUT=$O/nt timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0 --no-projection"
for c in 5 3 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $Q >> $O/bench_c$c.log 2>&1 || exit 1
done
