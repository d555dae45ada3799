#!/bin/bash
# Instruction mix of one bench step (rocprofv3 PMC passes, one run each):
#   bash tools/prof_mix.sh <tag> [extra bench args...]
set -u
R=${1:?tag}
shift
OUT=gpurun_out/$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -2 "$OUT/$name.log"; echo "== $name rc=$rc"; return $rc; }
Q="--steps 1 --warmup 0 --no-cpu-baseline --no-latency --unscreened-steps 0"
step trace 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python -u bench.py $Q "$@" || exit $?
step mix1 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT -d $OUT/mix1 -o run --output-format csv -- python -u bench.py $Q "$@" || exit $?
step mix2 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD -d $OUT/mix2 -o run --output-format csv -- python -u bench.py $Q "$@" || exit $?
echo done
