#!/bin/bash
# One measurement round on the GPU box: bench, kernel-trace stats, PMC passes.
# Every GPU step has its own time limit; stop at the first abnormal exit.
#   bash tools/prof_round.sh <tag> [extra bench args...]
set -u
R=${1:?round tag}
shift
OUT=gpurun_out/$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -3 "$OUT/$name.log"; echo "== $name rc=$rc"; return $rc; }
Q="--no-cpu-baseline --no-latency --unscreened-steps 0 --no-projection --no-other-configs --no-agreement"
step bench 400 python -u bench.py "$@" || exit $?
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python -u bench.py "$@" --steps 3 --warmup 1 $Q || exit $?
step pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python -u bench.py "$@" --steps 1 --warmup 3 $Q || exit $?
step pmc_write 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python -u bench.py "$@" --steps 1 --warmup 3 $Q || exit $?
step pmc_valu 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_valu -o run --output-format csv -- python -u bench.py "$@" --steps 1 --warmup 3 $Q || exit $?
echo done
