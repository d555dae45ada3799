# kernel-trace summary of a short config-3 bench (index build included once)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --unscreened-steps 0 > gpurun_out/c3prof.log 2>&1
echo traced
