"""Multi-GPU suggestion rounds: one process per GPU, candidates sharded by
global index, one collective per round.

Each rank scores candidates [rank*C, (rank+1)*C) of every label (the Philox
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
