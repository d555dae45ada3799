# round-4: k_bx_table with the next record batch prefetched (product) vs HEAD
# before it (var_r4pre2): winners, kernel-trace averages at configs 3 and 5
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4pre2.so timeout -k 10 200 python -u tools/ab_winners.py $O/pre.npz >> $O/ab.log 2>&1 || exit 1
python tools/ab_winners.py --compare $O/pre.npz $O/prod.npz >> $O/ab.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-projection --no-other-configs --no-agreement --unscreened-steps 0"
for v in prod r4pre2; do
  if [ $v = prod ]; then V=""; else V=tools/var_$v.so; fi
  for c in 3 5; do
    HYPEROPT_AMD_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_c$c -o run --output-format csv -- python -u bench.py --config $c $Q > $O/${v}_c$c.log 2>&1 || exit 1
  done
done
