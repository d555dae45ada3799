# round-4: k_hot_bx at R = 6 (no VGPR spills) vs the product R = 8: time and HBM traffic
set -o pipefail
O=gpurun_out/r4aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 1 --warmup 3 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in prod hot6; do
  if [ $v = prod ]; then V=""; else V=tools/var_$v.so; fi
  HYPEROPT_AMD_VARIANT=$V timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE -d $O/${v}_fetch -o run --output-format csv -- python -u bench.py $Q > $O/${v}_fetch.log 2>&1 || exit 1
  HYPEROPT_AMD_VARIANT=$V timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE -d $O/${v}_write -o run --output-format csv -- python -u bench.py $Q > $O/${v}_write.log 2>&1 || exit 1
  HYPEROPT_AMD_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_trace -o run --output-format csv -- python -u bench.py $Q --steps 3 --warmup 1 > $O/${v}_trace.log 2>&1 || exit 1
done
