# round-4: a label-shard-sized step (config 3 at 4 labels) under the runtime
# trace -- where a shard's fixed latency goes (kernels vs API calls vs gaps)
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
timeout -k 10 200 python -u bench.py --labels 4 $Q > $O/bench4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace --stats -d $O/rt -o run --output-format csv -- python -u bench.py --labels 4 $Q > $O/rt.log 2>&1
