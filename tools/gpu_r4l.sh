# round-4: per-wave hot listing buffers (product) against the per-tile flush
# (var_r4flush); the known labels' argsorts under the first build (early
# orders) on and off; the deferred-round and fmin-loop tests; stall counters
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4flush.so timeout -k 10 200 python -u tools/ab_winners.py $O/flush.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/flush.npz $O/prod.npz >> $O/ab.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_fmin_loop.py > $O/pytest.log 2>&1 || exit 1
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in "1" "0" "1" "0"; do
  timeout -k 10 200 python -u bench.py $Q --early-orders $v >> $O/bench_early$v.log 2>&1 || exit 1
done
HYPEROPT_AMD_VARIANT=tools/var_r4flush.so timeout -k 10 200 python -u bench.py $Q --early-orders 0 >> $O/bench_flush.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_stall -o run --output-format csv -- python -u bench.py $Q --steps 1 --warmup 3 > $O/pmc_stall.log 2>&1
