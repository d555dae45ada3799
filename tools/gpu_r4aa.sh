# round-4: mode-mask test; k_bx_table at 2 chains (var_bx2) and at <= 128 VGPRs (var_bxlb4), configs 3 and 5
set -o pipefail
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mode_mask.py > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in prod bx2 bxlb4; do
  if [ $v = prod ]; then V=""; else V=tools/var_$v.so; fi
  for c in 3 5; do
    HYPEROPT_AMD_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_c$c -o run --output-format csv -- python -u bench.py --config $c $Q > $O/${v}_c$c.log 2>&1 || exit 1
  done
done
