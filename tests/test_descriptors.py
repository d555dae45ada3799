"""north_star's partition (parallel.DescriptorExchange):
label shards build the posteriors and their expansion index, one all-gather
shares them (tpe_export_posterior / tpe_import_posterior), candidate shards
score the round, broadcast_best's merge (tpe.py:769-778) picks the winners.

CPU: the exchange's host logic over gloo with a stub engine (blob sizes,
slots, offsets, label lists, candidate slices, the merge).  GPU: the
imported posterior's rounds against one engine that built every label, bit
for bit -- whole rounds, candidate slices merged, batched rounds -- for the
mixed (config 3 / 5), conditional (config 4) and Hartmann (config 2)
spaces -- at 8 shards too, where some shards hold no dense label (no
index: the blob carries none, the import keeps the others') -- and a
two-rank gloo run of the whole exchange."""
import os
import socket

import numpy as np
import pytest

from hyperopt_amd.engine import RESULT_DTYPE


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


C_STUB = 1000


def _target(label, rnd):
    return (label * 37 + rnd * 11) % C_STUB


class _StubEngine(object):
    """Blob bytes = a rank pattern; a slice's winner = its candidate
    closest to a per-(round, label) target."""

    def __init__(self, rank, n_labels):
        self.rank, self.L = rank, n_labels
        self.imported = None

    def set_option(self, name, value):
        pass

    def export_size(self):
        return 1000 + 333 * self.rank

    def export_posterior(self, d_out):
        import torch
        n = self.export_size()
        d_out[:n] = (torch.arange(n) * (self.rank + 3) % 251).to(torch.uint8)
        return n

    def import_posterior(self, d_blobs, part_off, part_labels):
        self.imported = (d_blobs.numel(), [int(o) for o in part_off], [list(p) for p in part_labels],
                         [bytes(d_blobs[o:o + 1000 + 333 * r].cpu().numpy()) for r, o in enumerate(part_off)])

    def _labels(self):
        return self.L

    def suggest_batch(self, seed, rounds, n, cand_offset=0):
        out = np.zeros((len(rounds), self.L), dtype=RESULT_DTYPE)
        cand = np.arange(cand_offset, cand_offset + n)
        for i, r in enumerate(rounds):
            for l in range(self.L):
                d = np.abs(cand - _target(l, r))
                k = int(np.argmin(d))
                out[i, l]['index'] = cand[k]
                out[i, l]['score'] = -float(d[k])
                out[i, l]['value'] = cand[k] * 0.5
                out[i, l]['label'] = l
        return out


def _stub_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.parallel import DescriptorExchange
        shards = [[0, 3, 4], [1, 2, 5, 6]]
        eng = _StubEngine(rank, 7)
        x = DescriptorExchange(eng, shards, rank)
        sizes = x.share()
        res = x.round(5, [3, 4], C_STUB)
        q.put((rank, sizes, eng.imported, x.slice(C_STUB), res.tobytes()))
    finally:
        dist.destroy_process_group()


def test_descriptor_exchange_gloo_world2():
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stub_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, sizes, imported, sl, res = q.get(timeout=120)
        got[r] = (sizes, imported, sl, res)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        sizes, (total, offs, labels, parts), sl, res = got[r]
        assert sizes == [1000, 1333]
        assert offs == [0, 1536] and total == 2 * 1536       # 256-byte slots of the largest blob
        assert labels == [[0, 3, 4], [1, 2, 5, 6]]
        for k in (0, 1):
            n = 1000 + 333 * k
            assert parts[k] == bytes((np.arange(n) * (k + 3) % 251).astype(np.uint8))
        assert sl == ((0, 500) if r == 0 else (500, 500))
        out = np.frombuffer(res, dtype=RESULT_DTYPE).reshape(2, 7)
        for i, rnd in enumerate((3, 4)):
            assert list(out[i]['index']) == [_target(l, rnd) for l in range(7)]
    assert got[0][3] == got[1][3]


# ---------------------------------------------------------------- GPU

def _opts(eng, value_only=0):
    eng.set_option('value_only', value_only)


def _shard_blobs(hist, shards, n, C, dev=0):
    """Each shard's engine built through FminLoop (its labels, their space
    streams, the index queued for rounds of C), exported; the blobs packed
    in 256-byte slots of one device tensor."""
    import torch
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.parallel import _align
    from hyperopt_amd.workloads import FminLoop
    blobs = []
    for sh in shards:
        e = Engine(dev)
        try:
            _opts(e)
            lp = FminLoop(hist, label_ids=sh)
            lp.advance(e, n, n_candidates=C)
            b = torch.empty(e.export_size(), dtype=torch.uint8, device='cuda')
            assert e.export_posterior(b) == b.numel()
            blobs.append(b)
        finally:
            e.close()
    slot = max(_align(b.numel()) for b in blobs)
    allb = torch.zeros(slot * len(blobs), dtype=torch.uint8, device='cuda')
    for k, b in enumerate(blobs):
        allb[k * slot:k * slot + b.numel()] = b
    return allb, [k * slot for k in range(len(blobs))]


def _reference(hist, n, C, calls):
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop
    e = Engine(0)
    try:
        _opts(e)
        FminLoop(hist).advance(e, n, n_candidates=C)
        return [np.ascontiguousarray(f(e)).tobytes() for f in calls]
    finally:
        e.close()


def _space(name):
    from hyperopt_amd.workloads import conditional_history, hartmann_history, mixed_history
    if name == 'mixed32':
        return mixed_history(32, 6000, seed=3), 5990
    if name == 'conditional':
        return conditional_history(3000, seed=1), 2990
    return hartmann_history(1500, seed=4), 1490


@pytest.mark.gpu
@pytest.mark.parametrize('space,world', [('mixed32', 2), ('mixed32', 3), ('conditional', 2), ('hartmann', 2),
                                         ('conditional', 8), ('mixed32', 8)])
def test_imported_posterior_rounds_match_one_engine(space, world):
    from hyperopt_amd.engine import Engine, merge_results
    from hyperopt_amd.parallel import label_shards
    hist, n = _space(space)
    C = 1 << 18
    shards = label_shards(hist.labels, world)
    calls = [lambda e: e.suggest(42, C, round=9),
             lambda e: e.suggest_batch(7, list(range(300, 364)), 24)]
    want = _reference(hist, n, C, calls)
    allb, offs = _shard_blobs(hist, shards, n, C)
    e = Engine(0)
    try:
        _opts(e)
        e.import_posterior(allb, offs, shards)
        assert e._labels() == len(hist.labels)
        got = [np.ascontiguousarray(f(e)).tobytes() for f in calls]
        # candidate slices of the whole round, merged by broadcast_best's order
        parts = []
        for r in range(world):
            lo, hi = C * r // world, C * (r + 1) // world
            parts.append(e.suggest(42, hi - lo, round=9, cand_offset=lo))
        merged = merge_results(np.stack(parts))
    finally:
        e.close()
    assert got[0] == want[0], 'whole round on the imported posterior'
    assert got[1] == want[1], 'batched rounds on the imported posterior'
    w = np.frombuffer(want[0], dtype=RESULT_DTYPE)
    assert np.array_equal(merged['index'], w['index'])
    assert merged['value'].tobytes() == w['value'].tobytes()
    assert merged['score'].tobytes() == w['score'].tobytes()


@pytest.mark.gpu
def test_import_refuses_bad_parts():
    import torch
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.parallel import label_shards
    hist, n = _space('hartmann')
    shards = label_shards(hist.labels, 2)
    allb, offs = _shard_blobs(hist, shards, n, 1 << 12)
    e = Engine(0)
    try:
        with pytest.raises(Exception, match='permutation'):
            e.import_posterior(allb, offs, [shards[0], shards[0]])
        with pytest.raises(Exception, match='label count|posterior blob'):
            e.import_posterior(allb, offs, [shards[0] + shards[1][:1], shards[1][1:]])
        with pytest.raises(Exception, match='truncated|offset'):
            e.import_posterior(allb[:offs[1] + 256], offs, shards)
        junk = torch.zeros_like(allb)
        with pytest.raises(Exception, match='posterior blob'):
            e.import_posterior(junk, offs, shards)
    finally:
        e.close()


def _gpu_rank_worker(rank, world, port, q):
    """One rank of the descriptor exchange on the GPU (gloo: the blobs and
    winners staged through host tensors): build its shard, share, score its
    candidate slice, merge."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.engine import Engine
        from hyperopt_amd.parallel import DescriptorExchange, label_shards
        from hyperopt_amd.workloads import FminLoop
        hist, n = _space('mixed32')
        shards = label_shards(hist.labels, world)
        eng = Engine(0)
        x = DescriptorExchange(eng, shards, rank)
        loop = FminLoop(hist, label_ids=shards[rank])
        loop.advance(eng, n - 5)
        loop.advance(eng, n, n_candidates=1 << 18)
        x.share()
        res = x.round(42, [9], 1 << 18)
        eng.close()
        q.put((rank, np.ascontiguousarray(res[0]).tobytes()))
    except Exception:   # (reported, so the parent fails at once instead of waiting out its timeout)
        import traceback
        q.put((rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_descriptor_exchange_two_ranks_gpu():
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, a = q.get(timeout=100)
        assert isinstance(a, bytes), a
        got[r] = a
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hist, n = _space('mixed32')
    want = np.frombuffer(_reference(hist, n, 1 << 18, [lambda e: e.suggest(42, 1 << 18, round=9)])[0],
                         dtype=RESULT_DTYPE)
    for r in (0, 1):
        out = np.frombuffer(got[r], dtype=RESULT_DTYPE)
        assert np.array_equal(out['index'], want['index'])
        assert out['value'].tobytes() == want['value'].tobytes()
        assert out['score'].tobytes() == want['score'].tobytes()
    assert got[0] == got[1]
