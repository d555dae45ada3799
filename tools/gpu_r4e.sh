# round-4: device-merge diagnosis; k_hot_bx timing of the round-3 kernels
# (var_r4base), the rewritten k_hot_bx with the degree-2 exp (var_r4khot) and
# the product
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_parallel.py > $O/par.log 2>&1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement"
for v in tools/var_r4base.so tools/var_r4khot.so ""; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q > $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
