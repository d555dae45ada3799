#!/bin/bash
# Run one GPU step under its own time limit, log to gpurun_out/<name>.log.
# Exit codes: 0 ok, 1 test failure (continue allowed), anything else = stop.
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name: $*" 
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
tail -25 "gpurun_out/$name.log"
echo "== $name rc=$rc"
exit $rc
