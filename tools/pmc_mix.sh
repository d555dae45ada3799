#!/bin/bash
# One PMC pass of instruction-mix counters over a short warm bench (config 3):
#   bash tools/pmc_mix.sh <tag>
set -u
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--mode warm --steps 2 --warmup 1 --no-cpu-baseline --no-latency --unscreened-steps 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_mix -o run --output-format csv -- python -u bench.py $Q > $OUT/pmc_mix.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $OUT/pmc_mix2 -o run --output-format csv -- python -u bench.py $Q > $OUT/pmc_mix2.log 2>&1 || exit $?
echo done
