#!/bin/bash
# One measurement round on the GPU box: bench, kernel-trace stats, PMC passes.
# Every GPU step has its own time limit; stop at the first abnormal exit.
#   bash tools/prof_round.sh <tag> [extra bench args...]
# The passes (rocprofv3 collects what one pass can hold, so one pass each):
#   pmc_fetch / pmc_write   HBM bytes (FETCH_SIZE, WRITE_SIZE)
#   pmc_valu                VALU instructions, busy cycles, the launch's GPU cycles
#   pmc_mix                 VALU instructions by class (fp64 add/mul/fma/trans, int32/64, cvt)
#   pmc_mix32               fp32 classes (the same VALU total for the remainder)
#   pmc_stall               where the waves' cycles go (issue stalls, waits, LDS / scalar / VALU)
# tools/pmc_summary.py turns them into profiles/<tag>_pmc_summary.json.
set -u
R=${1:?round tag}
shift
OUT=gpurun_out/$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -3 "$OUT/$name.log"; echo "== $name rc=$rc"; return $rc; }
Q="--no-cpu-baseline --no-latency --unscreened-steps 0 --no-projection --no-other-configs --no-agreement"
pmc() { local name=$1; shift; step $name 150 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python -u bench.py $ARGS --steps 1 --warmup 3 $Q; }
ARGS="$*"
step bench 400 python -u bench.py "$@" || exit $?
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python -u bench.py "$@" --steps 3 --warmup 1 $Q || exit $?
pmc pmc_fetch FETCH_SIZE || exit $?
pmc pmc_write WRITE_SIZE || exit $?
pmc pmc_valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
pmc pmc_mix SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE || exit $?
pmc pmc_mix32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit $?
pmc pmc_stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE || exit $?
echo done
