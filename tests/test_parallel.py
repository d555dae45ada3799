"""The cross-rank exchanges (hyperopt_amd/parallel.py) with the gloo
backend, world_size 2: every rank ends with the broadcast_best merge of all
ranks' winners (candidate shards) or with every rank's rounds in order
(new_id shards) -- on CPU with synthetic rows, and on the GPU box with real
engine shards (two ranks sharing the card) against one unsharded engine."""
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
        from hyperopt_amd.parallel import exchange_winners, gather_rounds
        out = exchange_winners(_rank_results(rank))
        rows = np.stack([_rank_results(rank), _rank_results(rank + 10)])   # 2 rounds per rank
        q.put((rank, out.tobytes(), gather_rounds(rows).tobytes()))
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
    got, gathered = {}, {}
    for _ in procs:
        r, a, b = q.get(timeout=120)
        got[r], gathered[r] = a, b
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rounds = np.stack([_rank_results(0), _rank_results(10), _rank_results(1), _rank_results(11)])
    for r in (0, 1):
        g = np.frombuffer(gathered[r], dtype=RESULT_DTYPE).reshape(4, -1)
        assert np.array_equal(g['index'], rounds['index'])
    want = merge_results(np.stack([_rank_results(0), _rank_results(1)]))
    for r in (0, 1):
        out = np.frombuffer(got[r], dtype=RESULT_DTYPE)
        assert np.array_equal(out['index'], want['index'])
        assert out['index'][0] == 0          # tie -> rank 0's lower global index
        assert out['index'][1] == 1001       # NaN on rank 1 wins
    assert np.array_equal(np.frombuffer(got[0], dtype=RESULT_DTYPE)['index'],
                          np.frombuffer(got[1], dtype=RESULT_DTYPE)['index'])


def _engine_worker(rank, world, port, q):
    """One rank of a config-3-shaped run on the GPU: its candidate shard
    (global offset rank * C/world) and its share of batched new_ids."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.engine import Engine
        from hyperopt_amd.parallel import exchange_winners, gather_rounds
        from hyperopt_amd.workloads import mixed_history
        hist = mixed_history(16, 4000, seed=2)
        eng = Engine(0)
        eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
        eng.set_option('whole_rounds', 128)     # 128 new_ids over the two ranks
        C = 1 << 18
        mine = eng.suggest(42, C // world, round=9, cand_offset=rank * (C // world))
        merged = exchange_winners(mine)
        ids = list(range(500 + rank * 64, 500 + (rank + 1) * 64))
        rows = gather_rounds(eng.suggest_batch(7, ids, 24))
        eng.set_option('whole_rounds', 0)
        eng.close()
        q.put((rank, merged.tobytes(), rows.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_shards_gloo_world2():
    import multiprocessing as mp
    from hyperopt_amd.engine import RESULT_DTYPE, Engine
    from hyperopt_amd.workloads import mixed_history
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, a, b = q.get(timeout=200)
        got[r] = (a, b)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hist = mixed_history(16, 4000, seed=2)
    eng = Engine(0)
    eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
    want = eng.suggest(42, 1 << 18, round=9)
    want_rows = eng.suggest_batch(7, list(range(500, 628)), 24)
    eng.close()
    for r in (0, 1):
        merged = np.frombuffer(got[r][0], dtype=RESULT_DTYPE)
        rows = np.frombuffer(got[r][1], dtype=RESULT_DTYPE).reshape(want_rows.shape)
        for f in ('index', 'value', 'lpdf_below', 'lpdf_above'):
            assert np.array_equal(merged[f], want[f]), f
            assert np.array_equal(rows[f], want_rows[f]), f


def test_label_shards_partition():
    from hyperopt_amd.parallel import label_cost, label_shards
    from hyperopt_amd.workloads import mixed_space
    labels = mixed_space(32)
    for world in (1, 2, 3, 4, 8, 16):
        sh = label_shards(labels, world)
        assert sh == label_shards(labels, world)          # every rank computes the same
        assert sorted(i for s in sh for i in s) == list(range(32))
        assert all(s == sorted(s) and s for s in sh)
        load = [sum(label_cost(labels[i][1]) for i in s) for s in sh]
        # LPT: no shard exceeds the mean by more than the largest label cost
        assert max(load) <= sum(load) / world + 1.0
    with pytest.raises(ValueError):
        label_shards(labels[:3], 4)


def _label_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.parallel import gather_labels
        shards = [[0, 2, 5], [1, 3, 4, 6]]
        res = _rank_results(rank, n_labels=len(shards[rank]))
        res['index'] = np.array(shards[rank]) * 10 + rank
        rows = np.stack([res, res])                           # two rounds
        q.put((rank, gather_labels(res, shards, rank).tobytes(),
               gather_labels(rows, shards, rank).tobytes()))
    finally:
        dist.destroy_process_group()


def test_gather_labels_gloo_world2():
    import multiprocessing as mp
    from hyperopt_amd.engine import RESULT_DTYPE
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_label_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, a, b = q.get(timeout=120)
        got[r] = (a, b)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owner = [0, 1, 0, 1, 1, 0, 1]
    for r in (0, 1):
        out = np.frombuffer(got[r][0], dtype=RESULT_DTYPE)
        assert list(out['index']) == [10 * l + owner[l] for l in range(7)]
        assert list(out['label']) == list(range(7))
        rows = np.frombuffer(got[r][1], dtype=RESULT_DTYPE).reshape(2, 7)
        assert rows[0].tobytes() == out.tobytes() == rows[1].tobytes()   # (NaN scores: bytes)
    assert got[0] == got[1]


def _label_engine_worker(rank, world, port, q):
    """One rank of a label-sharded fmin step on the GPU: its labels' history,
    posterior and rounds (FminLoop label_ids), winners all-gathered."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.engine import Engine
        from hyperopt_amd.parallel import gather_labels, label_shards
        from hyperopt_amd.workloads import FminLoop, mixed_history
        hist = mixed_history(16, 4000, seed=2)
        shards = label_shards(hist.labels, world)
        eng = Engine(0)
        loop = FminLoop(hist, label_ids=shards[rank])
        loop.advance(eng, 3990)
        loop.advance(eng, 3995, n_candidates=1 << 18)
        one = gather_labels(eng.suggest(42, 1 << 18, round=9), shards, rank)
        rows = gather_labels(eng.suggest_batch(7, list(range(500, 628)), 24), shards, rank)
        eng.close()
        q.put((rank, one.tobytes(), rows.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_label_shards_gloo_world2():
    """Label-sharded ranks (bench.py's default N > 1 partition) end with the
    winners of one engine holding every label, bit for bit."""
    import multiprocessing as mp
    from hyperopt_amd.engine import RESULT_DTYPE, Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_label_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, a, b = q.get(timeout=200)
        got[r] = (a, b)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hist = mixed_history(16, 4000, seed=2)
    eng = Engine(0)
    loop = FminLoop(hist)
    loop.advance(eng, 3995)
    want = eng.suggest(42, 1 << 18, round=9)
    want_rows = eng.suggest_batch(7, list(range(500, 628)), 24)
    eng.close()
    for r in (0, 1):
        assert got[r][0] == want.tobytes()
        assert got[r][1] == np.ascontiguousarray(want_rows).tobytes()


def _xch_worker(rank, world, port, q):
    """DeviceExchange's collective + assembly on host tensors (gloo): the
    config-5 shape -- 4096 new_ids x a rank's labels (label shards: 64 and
    64 of 128), 2048 of the 4096 new_ids (rounds), and candidate shards."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd.engine import RESULT_DTYPE
        from hyperopt_amd.parallel import DeviceExchange
        from hyperopt_amd.workloads import mixed_space
        from hyperopt_amd.parallel import label_shards
        shards = label_shards(mixed_space(128), world)
        nr = 4096
        L = len(shards[rank])
        res = np.zeros((nr, L), dtype=RESULT_DTYPE)
        res['index'] = (np.arange(nr)[:, None] * 1000 + np.array(shards[rank])[None]) * 10 + rank
        res['value'] = res['index'] * 0.5
        raw = torch.from_numpy(np.ascontiguousarray(res).view(np.uint8).reshape(-1))
        out_l = DeviceExchange(None, 'labels', shards=shards, rank=rank).exchange(raw, nr, L)
        half = np.zeros((2048, 128), dtype=RESULT_DTYPE)
        half['index'] = rank * 2048 + np.arange(2048)[:, None]
        raw = torch.from_numpy(np.ascontiguousarray(half).view(np.uint8).reshape(-1))
        out_r = DeviceExchange(None, 'rounds', rank=rank).exchange(raw, 2048, 128)
        cand = np.stack([_rank_results(rank), _rank_results(rank + 10)])
        raw = torch.from_numpy(np.ascontiguousarray(cand).view(np.uint8).reshape(-1))
        out_c = DeviceExchange(None, 'candidates', rank=rank).exchange(raw, 2, cand.shape[1])
        q.put((rank, out_l.tobytes(), out_r.tobytes(), out_c.tobytes()))
    finally:
        dist.destroy_process_group()


def test_device_exchange_gloo_world2_config5_shapes():
    """the device-resident exchange's collective and
    assembly at world size 2 with config-5-shaped payloads (4096 rounds x
    64 labels per rank, label shards; 2048 rounds x 128 labels per rank, new_id
    shards) and candidate shards merged in the broadcast_best order."""
    import multiprocessing as mp
    from hyperopt_amd.engine import RESULT_DTYPE, merge_results
    from hyperopt_amd.parallel import label_shards
    from hyperopt_amd.workloads import mixed_space
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, a, b, c = q.get(timeout=180)
        got[r] = (a, b, c)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = label_shards(mixed_space(128), 2)
    owner = np.zeros(128, dtype=np.int64)
    for r, sh in enumerate(shards):
        owner[sh] = r
    want_l = (np.arange(4096)[:, None] * 1000 + np.arange(128)[None]) * 10 + owner[None]
    want_c = merge_results(np.stack([np.stack([_rank_results(0), _rank_results(10)]).reshape(-1),
                                     np.stack([_rank_results(1), _rank_results(11)]).reshape(-1)]))
    for r in (0, 1):
        out_l = np.frombuffer(got[r][0], dtype=RESULT_DTYPE).reshape(4096, 128)
        assert np.array_equal(out_l['index'], want_l)
        assert np.array_equal(out_l['label'][0], np.arange(128))
        out_r = np.frombuffer(got[r][1], dtype=RESULT_DTYPE).reshape(4096, 128)
        assert np.array_equal(out_r['index'][:, 0], np.arange(4096))
        out_c = np.frombuffer(got[r][2], dtype=RESULT_DTYPE).reshape(-1)
        assert np.array_equal(out_c['index'], want_c['index'])
    assert got[0] == got[1]


def _nccl_world1_worker(port, q):
    """DeviceExchange on the GPU under RCCL at world size 1 (a one-GPU box
    cannot hold two RCCL ranks): results written to a device buffer by the
    engine, all-gathered device to device, candidate shards merged on the GPU
    -- against the engine's host results."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1)
    try:
        from hyperopt_amd.engine import Engine, RESULT_DTYPE
        from hyperopt_amd.parallel import DeviceExchange
        from hyperopt_amd.workloads import mixed_history
        hist = mixed_history(16, 4000, seed=2)
        eng = Engine(0)
        eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
        out = {}
        for mode in ('candidates', 'rounds', 'labels'):
            x = DeviceExchange(eng, mode, shards=[list(range(16))], rank=0)
            out[mode] = (x.round(42, [9], 1 << 16)[0].tobytes(),
                         x.round(7, list(range(500, 628)), 24).tobytes())
        out['host'] = (eng.suggest(42, 1 << 16, round=9).tobytes(),
                       eng.suggest_batch(7, list(range(500, 628)), 24).tobytes())
        # the device merge against the host merge over 3 parts
        a = eng.suggest(1, 4096, round=1, cand_offset=0)
        b = eng.suggest(1, 4096, round=1, cand_offset=4096)
        c = eng.suggest(1, 4096, round=1, cand_offset=8192)
        parts = np.ascontiguousarray(np.stack([a, b, c]))
        d_parts = torch.from_numpy(parts.view(np.uint8).reshape(-1)).cuda()
        d_out = torch.empty(len(a) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device='cuda')
        eng.merge_results_device(d_parts, 3, len(a), d_out)
        out['merge'] = d_out.cpu().numpy().tobytes()
        out['parts'] = parts.tobytes()
        out['d_parts'] = d_parts.cpu().numpy().tobytes()
        from hyperopt_amd.engine import merge_results
        out['merge_host'] = np.ascontiguousarray(merge_results(parts)).tobytes()
        eng.close()
        q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_device_exchange_rccl_world1():
    import multiprocessing as mp
    from hyperopt_amd.engine import merge_results, RESULT_DTYPE
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    def diff(a, b):
        a = np.frombuffer(a, dtype=RESULT_DTYPE)
        b = np.frombuffer(b, dtype=RESULT_DTYPE)
        return [(int(i), a[i]['index'], b[i]['index'], a[i]['value'], b[i]['value'], a[i]['score'],
                 b[i]['score']) for i in range(len(a)) if a[i].tobytes() != b[i].tobytes()][:5]
    for mode in ('candidates', 'rounds', 'labels'):
        assert out[mode][0] == out['host'][0], (mode, diff(out[mode][0], out['host'][0]))
        assert out[mode][1] == out['host'][1], (mode, diff(out[mode][1], out['host'][1]))
    assert out['d_parts'] == out['parts']
    if out['merge'] != out['merge_host']:
        parts = np.frombuffer(out['parts'], dtype=RESULT_DTYPE).reshape(3, -1)
        a = np.frombuffer(out['merge'], dtype=RESULT_DTYPE)
        b = np.frombuffer(out['merge_host'], dtype=RESULT_DTYPE)
        bad = [j for j in range(len(a)) if a[j].tobytes() != b[j].tobytes()]
        raise AssertionError('device merge differs at %s: device %s host %s parts %s' % (
            bad, a[bad[0]], b[bad[0]], parts[:, bad[0]]))
