#!/bin/bash
# fresh-posterior bench (config 3) + kernel trace of the same command
set -u
OUT=gpurun_out/${1:-fresh}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-latency --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -c 3000 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-latency --no-cpu-baseline --unscreened-steps 0 --no-projection > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
echo done
