# per-kernel time of engine variants (tools/var_*.so from tools/build_variant.py),
# each loaded through the explicit opt-in HYPEROPT_AMD_VARIANT; the product
# library is never replaced
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base bm; do
  if [ "$v" = base ]; then unset HYPEROPT_AMD_VARIANT; else export HYPEROPT_AMD_VARIANT=tools/var_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vt_$v -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --unscreened-steps 0 > gpurun_out/vt_$v.log 2>&1
  echo "$v: $(grep k_hot_bx gpurun_out/vt_$v/run_kernel_stats.csv | cut -d, -f4)"
done
