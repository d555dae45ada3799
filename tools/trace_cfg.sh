#!/bin/bash
# kernel trace of a short bench run: bash tools/trace_cfg.sh <tag> <bench args...>
set -u
OUT=gpurun_out/${1:?tag}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python -u bench.py "$@" --no-latency --no-cpu-baseline --unscreened-steps 0 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python tools/kstats.py $OUT/trace/run_kernel_stats.csv 20
