# round-4 final (after k_split registers, runs beside the index, armed prepare): default line + profile set
set -o pipefail
mkdir -p gpurun_out/r4aw
timeout -k 10 420 python -u bench.py > gpurun_out/r4aw/bench_default.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4aw/smoke.log 2>&1 || exit 1
bash tools/prof_round.sh r4aw --steps 5 --warmup 2 --no-other-configs --no-agreement
