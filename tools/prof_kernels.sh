#!/bin/bash
# Kernel-trace stats of short bench runs (one per config) on the GPU box:
#   bash tools/prof_kernels.sh <tag> <config> [<config> ...]
# writes gpurun_out/<tag>_c<config>/ (rocprofv3 --kernel-trace --stats).
set -u
R=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in "$@"; do
    OUT=gpurun_out/${R}_c$c
    mkdir -p $OUT
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
        python -u bench.py --config $c --steps 3 --warmup 1 --no-latency --no-cpu-baseline \
        --unscreened-steps 0 > $OUT/bench.log 2>&1 || exit $?
    echo "== config $c done"
done
