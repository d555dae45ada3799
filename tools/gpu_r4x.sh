# round-4: persistent k_screen_hot (work items, table staged once per
# workgroup) against HEAD before it (var_r4pre3): winners, the screen tests,
# kernel-trace averages
set -o pipefail
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4pre3.so timeout -k 10 200 python -u tools/ab_winners.py $O/pre.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/pre.npz $O/prod.npz >> $O/ab.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_screen.py tests/test_fmin_loop.py tests/test_value_only.py > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in prod r4pre3; do
  if [ $v = prod ]; then V=""; else V=tools/var_$v.so; fi
  HYPEROPT_AMD_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python -u bench.py $Q > $O/$v.log 2>&1 || exit 1
done
