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


def exchange_winners(res, group=None):
    """All-gather per-rank winners and merge; returns the merged winners."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return res
    res = np.ascontiguousarray(res, dtype=RESULT_DTYPE)
    raw = torch.from_numpy(res.view(np.uint8).copy())
    if dist.get_backend(group) == 'nccl':
        raw = raw.cuda()
    out = torch.empty(world * raw.numel(), dtype=torch.uint8, device=raw.device)
    dist.all_gather_into_tensor(out, raw, group=group)
    parts = out.cpu().numpy().view(RESULT_DTYPE).reshape((world,) + res.shape)
    return merge_results(parts.reshape(world, -1)).reshape(res.shape)


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
