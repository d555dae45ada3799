# per-kernel time of engine variants (tools/var_*.so, experiment macros)
# (build the variants first: cp hyperopt_amd/libhyperopt_tpe.so tools/var_base.so; python tools/build_variant.py bm TPE_EXP_BM_CHEAP)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base bm; do
  cp tools/var_$v.so hyperopt_amd/libhyperopt_tpe.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vt_$v -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --unscreened-steps 0 > gpurun_out/vt_$v.log 2>&1
  echo "$v: $(grep k_hot_bx gpurun_out/vt_$v/run_kernel_stats.csv | cut -d, -f4)"
done
