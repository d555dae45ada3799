"""The cross-rank winner exchange (hyperopt_amd/parallel.py) with the gloo
backend, world_size 2, on CPU: every rank ends with the broadcast_best merge
of all ranks' winners."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_results(rank, n_labels=7):
    from hyperopt_amd.engine import RESULT_DTYPE
    rng = np.random.RandomState(100 + rank)
    r = np.zeros(n_labels, dtype=RESULT_DTYPE)
    r['score'] = rng.normal(size=n_labels)
    r['score'][0] = 1.0              # tie on label 0 -> lower global index wins
    r['score'][1] = np.nan if rank == 1 else 5.0   # NaN beats everything
    r['index'] = rank * 1000 + np.arange(n_labels)
    r['value'] = rank + 0.5
    r['label'] = np.arange(n_labels)
    return r


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.parallel import exchange_winners
        out = exchange_winners(_rank_results(rank))
        q.put((rank, out.tobytes()))
    finally:
        dist.destroy_process_group()


def test_exchange_winners_gloo_world2():
    import multiprocessing as mp
    from hyperopt_amd.engine import RESULT_DTYPE, merge_results
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = merge_results(np.stack([_rank_results(0), _rank_results(1)]))
    for r in (0, 1):
        out = np.frombuffer(got[r], dtype=RESULT_DTYPE)
        assert np.array_equal(out['index'], want['index'])
        assert out['index'][0] == 0          # tie -> rank 0's lower global index
        assert out['index'][1] == 1001       # NaN on rank 1 wins
    assert np.array_equal(np.frombuffer(got[0], dtype=RESULT_DTYPE)['index'],
                          np.frombuffer(got[1], dtype=RESULT_DTYPE)['index'])
