#!/bin/bash
# GPU tests then the fresh-posterior bench + kernel trace (tools/fresh_probe.sh)
#   bash tools/gpu_round.sh <tag> [pytest -k expr]
set -u
T=${1:?tag}
K=${2:-}
mkdir -p gpurun_out/$T
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$T/gputest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
fi
rc=$?
tail -15 gpurun_out/$T/gputest.log
[ $rc -eq 0 ] || exit $rc
bash tools/fresh_probe.sh $T
