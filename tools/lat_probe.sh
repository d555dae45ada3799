# tpe.suggest latency (config 3, C = 24) and its kernel trace
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/latency_breakdown.py > gpurun_out/lat.log 2>&1
tail -25 gpurun_out/lat.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/latprof -o run --output-format csv -- python -u tools/latency_breakdown.py > gpurun_out/latprof.log 2>&1
echo traced
