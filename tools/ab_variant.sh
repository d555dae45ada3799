#!/bin/bash
# A/B: product library vs a variant (tools/var_<name>.so), bench screen ms
#   bash tools/ab_variant.sh <tag> <variant>
set -u
OUT=gpurun_out/$1${EXTRA:+_c}
mkdir -p $OUT
for v in prod $2 prod $2; do
  if [ $v = prod ]; then E=""; else E="tools/var_$v.so"; fi; export BENCH_SUBSET_REBUILD=${SUBSET:-1}
  HYPEROPT_AMD_VARIANT=$E timeout -k 10 200 python -u tools/bench_opts.py --steps 8 --warmup 2 --no-latency --no-cpu-baseline --no-projection --unscreened-steps 0 ${EXTRA:-} > $OUT/$v.log 2>&1 || exit 1
  python -c "
import json;l=[x for x in open('$OUT/$v.log') if x.startswith('{')][-1];j=json.loads(l);print('$v', round(j['ms_per_step'],3), j['step']['warm_round_ms'], j['screen']['screen_kernel_ms'], j['step']['expansion_index_ms'])"
done
