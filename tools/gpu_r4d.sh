# round-4: bench (default line: configs 2/4/5 legs, near-tie leg), then the GPU suite
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O/nt
timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit 1
NEAR_TIE_OUT=$O/nt timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
