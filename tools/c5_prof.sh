#!/bin/bash
# fresh-posterior lines of configs 2, 4, 5 and a kernel trace of config 5
set -u
T=${1:?tag}
OUT=gpurun_out/$T
bash tools/configs_fresh.sh $T || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace5 -o run --output-format csv -- python -u bench.py --config 5 --steps 3 --warmup 1 --no-latency --no-cpu-baseline --unscreened-steps 0 --no-projection > $OUT/trace5.log 2>&1 || { tail -30 $OUT/trace5.log; exit 1; }
echo done
