#!/bin/bash
# shard probes (one 8-way label shard, and all labels) + a kernel trace
#   bash tools/shard_prof.sh <tag> [shard]
set -u
OUT=gpurun_out/${1:-shard}
S=${2:-4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/shard_probe.py $S 20 > $OUT/probe.log 2>&1 || { tail -30 $OUT/probe.log; exit 1; }
timeout -k 10 200 python -u tools/shard_probe.py -1 20 > $OUT/probe_all.log 2>&1 || { tail -30 $OUT/probe_all.log; exit 1; }
cat $OUT/probe.log $OUT/probe_all.log
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/trace -o run --output-format csv -- python -u tools/shard_probe.py $S 10 > $OUT/trace.log 2>&1 || { tail -30 $OUT/trace.log; exit 1; }
echo done
