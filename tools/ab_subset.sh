mkdir -p gpurun_out/r3ae
for v in 1 0 1 0; do timeout -k 10 200 python -u -c "
import sys, runpy
import hyperopt_amd.posterior as P
P.SUBSET_REBUILD = bool($v)
sys.argv = ['bench.py', '--steps', '8', '--warmup', '2', '--no-latency', '--no-cpu-baseline', '--no-projection', '--unscreened-steps', '0']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r3ae/b$v.log 2>&1 || exit 1; python -c "
import json;l=[x for x in open('gpurun_out/r3ae/b$v.log') if x.startswith('{')][-1];j=json.loads(l);print('subset=$v', round(j['ms_per_step'],3), j['step']['warm_round_ms'], j['screen']['screen_kernel_ms'])"; done
