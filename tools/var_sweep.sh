# timing of engine variants (tools/var_*.so from tools/build_variant.py): each
# loaded through the explicit opt-in, the product library untouched
set -e
for v in bm norej; do
  HYPEROPT_AMD_VARIANT=tools/var_$v.so bash tools/q_sweep.sh | sed "s/^/$v: /"
done
bash tools/q_sweep.sh | sed "s/^/base: /"
