#!/bin/bash
# kernel trace of bench.py on a variant library (experiment): tools/trace_var.sh <tag> <variant> [bench args]
T=$1; V=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$T
export HYPEROPT_AMD_VARIANT=tools/var_$V.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/tr_$V -o run --output-format csv -- python -u bench.py "$@" > gpurun_out/$T/tr_$V.log 2>&1
