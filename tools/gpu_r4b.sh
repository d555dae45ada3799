# round-4 check: draws unchanged vs the previous commit (winners bit for
# bit), the whole GPU suite, then the bench
set -o pipefail
mkdir -p gpurun_out/r4b
export NEAR_TIE_OUT=gpurun_out/r4b
timeout -k 10 300 python -u tools/ab_winners.py gpurun_out/r4b/prod.npz > gpurun_out/r4b/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4base.so timeout -k 10 300 python -u tools/ab_winners.py gpurun_out/r4b/base.npz >> gpurun_out/r4b/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare gpurun_out/r4b/prod.npz gpurun_out/r4b/base.npz >> gpurun_out/r4b/ab.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r4b/pytest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r4b/bench.log 2>&1
