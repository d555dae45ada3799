# round-4 final: side families on in tpe.suggest and the bench -- whole GPU suite, smoke, default line + profile set
set -o pipefail
O=gpurun_out/r4bc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py > $O/bench_default.log 2>&1 || exit 1
bash tools/prof_round.sh r4bc --steps 5 --warmup 2 --no-other-configs --no-agreement
