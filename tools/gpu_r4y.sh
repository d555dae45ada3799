# round-4: k_hot_bx slots per thread (R = 8 product, 6, 4) and 6 workgroups per CU at R = 4
set -o pipefail
O=gpurun_out/r4y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in prod hot6 hot4 lb6; do
  if [ $v = prod ]; then V=""; else V=tools/var_$v.so; fi
  HYPEROPT_AMD_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python -u bench.py $Q > $O/$v.log 2>&1 || exit 1
done
