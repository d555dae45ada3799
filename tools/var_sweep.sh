# timing of engine variants (tools/var_*.so, experiment macros): swap each in, bench
# (build the variants first: cp hyperopt_amd/libhyperopt_tpe.so tools/var_base.so; python tools/build_variant.py bm TPE_EXP_BM_CHEAP)
set -e
for v in base bm norej; do
  cp tools/var_$v.so hyperopt_amd/libhyperopt_tpe.so
  bash tools/q_sweep.sh | sed "s/^/$v: /"
done
