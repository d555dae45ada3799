# round-4 final: default bench line, then the profile set (trace + PMC passes)
set -o pipefail
mkdir -p gpurun_out/r4ar
timeout -k 10 420 python -u bench.py > gpurun_out/r4ar/bench_default.log 2>&1 || exit 1
bash tools/prof_round.sh r4ar --steps 5 --warmup 2 --no-other-configs --no-agreement
