for d in 0 1 2 4 3 5 6 7; do echo "dbg $d"; TPE_BX_DBG=$d timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --unscreened-steps 0 > gpurun_out/dbg$d.log 2>&1 || exit 1; python3 -c "
import json
for l in open('gpurun_out/dbg$d.log'):
    if l.startswith('{'): d=json.loads(l); print(d['screen']['screen_kernel_ms'])"; done
