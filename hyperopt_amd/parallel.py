"""Multi-GPU suggestion rounds: one process per GPU, one collective per
round.  Two partitions of a round's (label, candidate) set:

* label shards (label_shards / gather_labels): rank r holds the labels of
  its shard -- their history columns, posterior, expansion index and every
  candidate of their rounds -- so the per-posterior work (rebuild, index)
  divides over the ranks like the candidates do.  Labels are independent in
  tpe.suggest (one build_posterior_wrapper + broadcast_best per label,
  tpe.py:678-692, 769-778) and each keeps its Philox stream, so the winners
  are the single-GPU winners; the all-gather carries 48 B per label.
* candidate shards (exchange_winners): rank r scores candidates
  [rank*C, (rank+1)*C) of every label, for spaces with fewer labels than
  ranks.
* descriptor exchange (DescriptorExchange): label shards for the posterior
  and index builds, then one all-gather of the built posteriors and
  candidate shards for the round -- north_star's partition.

Candidate shards: each rank scores candidates [rank*C, (rank+1)*C) of every label (the Philox
counter is the global index, so the union over ranks is exactly the
single-GPU candidate set).  The per-label winners (48 B x L) are
all-gathered -- over RCCL (`nccl` backend) on GPUs, gloo in the CPU tests --
and every rank merges them with the broadcast_best order (tpe.py:769-778:
larger score, NaN greatest, lowest global index), so all ranks hold the same
winners.
"""
import numpy as np

from .engine import RESULT_DTYPE, merge_results


def _all_gather_results(res, group):
    """(world,) + res.shape array of every rank's result records (one RCCL
    all-gather of the raw 48-byte records; gloo on CPU)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    res = np.ascontiguousarray(res, dtype=RESULT_DTYPE)
    raw = torch.from_numpy(res.view(np.uint8).reshape(-1))
    if dist.get_backend(group) == 'nccl':
        raw = raw.cuda(non_blocking=True)
    out = torch.empty(world * raw.numel(), dtype=torch.uint8, device=raw.device)
    dist.all_gather_into_tensor(out, raw, group=group)
    return out.cpu().numpy().view(RESULT_DTYPE).reshape((world,) + res.shape)


def all_gather_raw(raw, group=None):
    """One all-gather of a rank's raw result records (a contiguous uint8
    tensor: on the GPU under RCCL, on the CPU under gloo); returns the
    (world * nbytes,) tensor on the same device."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty(world * raw.numel(), dtype=torch.uint8, device=raw.device)
    dist.all_gather_into_tensor(out, raw.reshape(-1), group=group)
    return out


def _records(t, shape):
    return t.cpu().numpy().view(RESULT_DTYPE).reshape(shape)


def assemble_labels(gathered, lead, m, shards):
    """Label-shard assembly of an all-gather of padded [lead][m] record
    blocks (one per rank, in rank order): [lead][n_labels] in space order,
    `label` set to the space index."""
    world = len(shards)
    parts = gathered.reshape((world,) + tuple(lead) + (m,))
    n_labels = sum(len(sh) for sh in shards)
    out = np.zeros(tuple(lead) + (n_labels,), dtype=RESULT_DTYPE)
    for r, sh in enumerate(shards):
        out[..., sh] = parts[r][..., :len(sh)]
    out['label'] = np.arange(n_labels, dtype=np.int32)
    return out


class DeviceExchange(object):
    """Winners exchanged where they are computed: the
    engine leaves a round's results in a device buffer (tpe_suggest_batch_
    device), ONE all-gather moves every rank's buffer -- RCCL over xGMI,
    device to device -- candidate shards are merged on the GPU
    (tpe_merge_results_device), and only the final winners come to the host
    (tpe.suggest's documents need them there).  The round-2/3 path staged the
    records through host numpy, H2D, the collective and D2H every round.

    mode 'labels' (rank r holds shards[r]'s labels: records padded to the
    largest shard), 'candidates' (every rank the same rounds over its slice
    of the candidates: broadcast_best merge) or 'rounds' (rank r holds rounds
    [r n, (r + 1) n) of every label).  Under gloo (CPU rehearsals) the same
    gather runs on host tensors."""

    def __init__(self, engine, mode, shards=None, rank=0, group=None):
        import torch.distributed as dist
        if mode not in ('labels', 'candidates', 'rounds'):
            raise ValueError(mode)
        self.engine, self.mode, self.shards, self.rank, self.group = engine, mode, shards, rank, group
        self.world = dist.get_world_size(group)
        if mode == 'candidates' and engine is not None:
            # the shards' winners merge by score: a value-only round
            # (get_engine's default) leaves a certified cell without one
            engine.set_option('value_only', 0)
        self.device = dist.get_backend(group) == 'nccl'
        self._bufs = {}

    def _buf(self, key, nbytes):
        import torch
        b = self._bufs.get(key)
        if b is None or b.numel() < nbytes:
            b = self._bufs[key] = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
        return b[:nbytes]

    def round(self, seed, rounds, n_candidates, cand_offset=0):
        """Run this rank's share of the rounds and exchange: every rank
        returns [len(rounds) (x world for 'rounds')][n_labels] records."""
        import torch
        eng = self.engine
        nr = len(rounds)
        L = eng._labels()
        rec = RESULT_DTYPE.itemsize
        if self.device:
            raw = eng.suggest_batch_device(seed, rounds, n_candidates, self._buf('res', nr * L * rec),
                                           cand_offset=cand_offset)
        else:
            res = eng.suggest_batch(seed, rounds, n_candidates, cand_offset=cand_offset)
            raw = torch.from_numpy(np.ascontiguousarray(res).view(np.uint8).reshape(-1))
        return self.exchange(raw, nr, L)

    def exchange(self, raw, nr, L):
        """The collective and the assembly for raw = this rank's [nr][L]
        records as a uint8 tensor (device or host)."""
        import torch
        rec = RESULT_DTYPE.itemsize
        if self.mode == 'labels':
            m = max(len(sh) for sh in self.shards)
            if m != L:   # pad each round's block to the largest shard
                pad = (self._buf('pad', nr * m * rec) if raw.is_cuda
                       else torch.zeros(nr * m * rec, dtype=torch.uint8))
                pad.view(nr, m * rec)[:, :L * rec] = raw.view(nr, L * rec)
                raw = pad
            g = all_gather_raw(raw, self.group)
            return assemble_labels(_records(g, (-1,)), (nr,), m, self.shards)
        g = all_gather_raw(raw, self.group)
        if self.mode == 'rounds':
            return _records(g, (self.world * nr, L))
        if raw.is_cuda:   # candidates: the broadcast_best merge on the GPU
            out = self._buf('merged', nr * L * rec)
            self.engine.merge_results_device(g, self.world, nr * L, out)
            return _records(out, (nr, L))
        return merge_results(_records(g, (self.world, nr * L))).reshape(nr, L)


def _align(n, a=256):
    return (int(n) + a - 1) // a * a


class DescriptorExchange(object):
    """north_star's partition: the
    per-posterior work divides over the ranks like label shards -- rank r
    appends its labels' observations, rebuilds their posteriors and their
    expansion index (FminLoop over label_shards(...)[r]) -- and the rounds
    divide like candidate shards: share() exports this rank's posterior as
    one device blob (tpe_export_posterior), ONE all-gather over RCCL moves
    every rank's blob device to device, and every rank imports the whole
    space's posterior (tpe_import_posterior: each label's records and index,
    rebased, in space order); round() then scores candidates [r C/N, (r+1)
    C/N) of every label and the winners merge on the GPU with broadcast_best's
    order (DeviceExchange 'candidates').  Labels are independent in
    tpe.suggest (tpe.py:678-692) and each keeps its Philox stream, so the
    merged winners are one context's winners over the whole round.

    Two collectives per step beyond the winners' all-gather: the blob sizes
    (N int64) and the blobs (N x the largest, 256-byte slots)."""

    def __init__(self, engine, shards, rank, group=None, split='candidates'):
        import torch.distributed as dist
        if split not in ('candidates', 'rounds'):
            raise ValueError(split)
        self.engine, self.shards, self.rank, self.group = engine, shards, rank, group
        self.world = dist.get_world_size(group)
        if len(shards) != self.world:
            raise ValueError('%d label shards for %d ranks' % (len(shards), self.world))
        self.device = dist.get_backend(group) == 'nccl'
        self.split = split
        self.winners = DeviceExchange(engine, split, rank=rank, group=group)
        self._bufs = {}
        self.last_sizes = None

    def _buf(self, key, nbytes, dtype=None, device=None):
        import torch
        dev = torch.device(device or ('cuda' if self.device else 'cpu'))
        b = self._bufs.get(key)
        if b is None or b.numel() < nbytes or b.device.type != dev.type or (
                dev.index is not None and b.device.index != dev.index):
            b = self._bufs[key] = torch.empty(nbytes, dtype=dtype or torch.uint8, device=dev)
        return b[:nbytes]

    def share(self):
        """Export, all-gather, import: afterwards this rank's engine holds
        every label's posterior and index.  Returns the ranks' blob sizes.
        (Under gloo -- the CPU and one-GPU rehearsals -- the blobs are staged
        through host tensors around the collective.)"""
        import torch
        import torch.distributed as dist
        eng = self.engine
        # the engine's side: its GPU (a stub engine of the CPU tests: host)
        # (the engine's own card, not torch's current device: a rank need not
        # have called torch.cuda.set_device(engine.device) -- ADVICE r5)
        edev = (torch.device('cuda', int(getattr(eng, 'device', 0))) if torch.cuda.is_available()
                else torch.device('cpu'))
        sz = self._buf('size', 1, torch.int64)
        sz.fill_(eng.export_size())
        allsz = self._buf('sizes', self.world, torch.int64)
        dist.all_gather_into_tensor(allsz, sz, group=self.group)
        sizes = [int(v) for v in allsz.tolist()]
        slot = _align(max(sizes))
        blob = self._buf('blob', slot, device=edev)
        eng.export_posterior(blob)
        blobs = self._buf('blobs', self.world * slot, device=edev)
        if blob.device.type == ('cuda' if self.device else 'cpu'):   # (the collective's side)
            dist.all_gather_into_tensor(blobs, blob, group=self.group)
        else:
            staged = self._buf('staged', self.world * slot)
            dist.all_gather_into_tensor(staged, blob.to(staged.device), group=self.group)
            blobs.copy_(staged)
        eng.import_posterior(blobs, [r * slot for r in range(self.world)], self.shards)
        self.last_sizes = sizes
        return sizes

    def slice(self, n_candidates):
        """(cand_offset, count) of this rank's candidates of every label."""
        lo = n_candidates * self.rank // self.world
        return lo, n_candidates * (self.rank + 1) // self.world - lo

    def round(self, seed, rounds, n_candidates):
        """split 'candidates': this rank's slice of the rounds (n_candidates
        per label over all ranks); 'rounds' (batched new_ids, config 5): this
        rank's rounds whole.  Then the winners' exchange: [len(rounds) (x
        world for 'rounds')][n_labels] records."""
        if self.split == 'rounds':
            return self.winners.round(seed, rounds, n_candidates)
        off, n = self.slice(n_candidates)
        return self.winners.round(seed, rounds, n, cand_offset=off)


def exchange_winners(res, group=None):
    """All-gather per-rank winners of the SAME rounds (candidate shards) and
    merge them; every rank returns the merged winners."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return res
    parts = _all_gather_results(res, group)
    return merge_results(parts.reshape(world, -1)).reshape(np.shape(res))


def gather_rounds(res, group=None):
    """All-gather per-rank winners of DIFFERENT rounds (new_id shards, rank r
    holding rounds [r n, (r+1) n)); every rank returns all rounds in order."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return res
    parts = _all_gather_results(res, group)
    return parts.reshape((world * np.shape(res)[0],) + np.shape(res)[1:])


# relative cost of a label in a fresh-posterior step of a label shard,
# fitted to the one-GPU projection's shard times (r3ac: 3 dense + 1
# categorical 1.20 ms, 2 dense + 2 quantized 1.44 ms, 2 dense + 1 quantized
# + 2 categorical 1.33 ms): a dense label pays its share of the draw kernel
# and of the index, a quantized one the host's numpy argsort, its part of
# the ordered rebuild and its table round -- more than a dense one -- a
# categorical one its early-exit round
LABEL_COST = {'dense': 1.0, 'quantized': 1.5, 'categorical': 0.5}


def label_cost(kind, args=None):
    if kind in ('randint', 'categorical'):
        return LABEL_COST['categorical']
    if kind.startswith('q'):
        return LABEL_COST['quantized']
    return LABEL_COST['dense']


def label_shards(labels, world):
    """Partition of label indices over `world` ranks, longest processing
    time first (largest cost to the least-loaded rank; ties to the lower
    rank and label, so every rank computes the same partition); each shard
    in increasing label order."""
    if world > len(labels):
        raise ValueError('%d labels cannot fill %d label shards' % (len(labels), world))
    load = [0.0] * world
    shards = [[] for _ in range(world)]
    order = sorted(range(len(labels)), key=lambda i: (-label_cost(labels[i][1]), i))
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += label_cost(labels[i][1])
    return [sorted(sh) for sh in shards]


def gather_labels(res, shards, rank, group=None):
    """All-gather the winners of label shards: res[..., j] is this rank's
    result for label shards[rank][j]; every rank returns res[..., L] over all
    labels in space order, `label` set to the space index."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    n_labels = sum(len(sh) for sh in shards)
    m = max(len(sh) for sh in shards)
    res = np.asarray(res, dtype=RESULT_DTYPE)
    lead = res.shape[:-1]
    pad = np.zeros(lead + (m,), dtype=RESULT_DTYPE)
    pad['index'] = -1
    pad[..., :res.shape[-1]] = res
    parts = _all_gather_results(pad, group) if world > 1 else pad[None]
    out = np.zeros(lead + (n_labels,), dtype=RESULT_DTYPE)
    for r, sh in enumerate(shards):
        out[..., sh] = parts[r][..., :len(sh)]
    out['label'] = np.arange(n_labels, dtype=np.int32)
    return out


class ShardedSuggest(object):
    """Engine rounds over this rank's candidate shard + winner exchange."""

    def __init__(self, engine, group=None):
        import torch.distributed as dist
        self.engine = engine
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def suggest(self, seed, n_candidates_per_rank, round=0):
        res = self.engine.suggest(seed, n_candidates_per_rank, round=round,
                                  cand_offset=self.rank * n_candidates_per_rank)
        return exchange_winners(res, self.group) if self.world > 1 else res
