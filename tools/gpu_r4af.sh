# round-4: bench's multi-process path rehearsed with two gloo ranks sharing the one GPU
# (config 3 label shards, config 5 label shards, config 2 candidate shards)
set -o pipefail
O=gpurun_out/r4af
mkdir -p $O
for c in 3 5 2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$c bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --config $c > $O/n2_c$c.log 2>&1 || exit 1
done
