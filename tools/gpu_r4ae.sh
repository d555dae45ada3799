# round-4: config 5's step breakdown and kernel stats
set -o pipefail
O=gpurun_out/r4ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-other-configs --no-agreement --unscreened-steps 0 --no-projection"
timeout -k 10 200 python -u bench.py --config 5 $Q > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python -u bench.py --config 5 $Q --steps 3 --warmup 1 > $O/trace.log 2>&1
