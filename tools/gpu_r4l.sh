# round-4: per-wave hot listing buffers (product) against the per-tile flush (var_r4flush)
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4flush.so timeout -k 10 200 python -u tools/ab_winners.py $O/flush.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/flush.npz $O/prod.npz >> $O/ab.log 2>&1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in "" tools/var_r4flush.so "" tools/var_r4flush.so; do
  HYPEROPT_AMD_VARIANT=$v timeout -k 10 200 python -u bench.py $Q >> $O/bench_$(basename "${v:-prod}" .so).log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_stall -o run --output-format csv -- python -u bench.py $Q --steps 1 --warmup 3 > $O/pmc_stall.log 2>&1
