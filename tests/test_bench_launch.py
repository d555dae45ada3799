"""bench.py --gpus N: N > 1 without a torchrun
environment starts N rank processes under torch.distributed.run, every rank
checks that the process group is the N ranks it was asked for, and a node
with fewer GPUs than ranks is refused with a non-zero exit instead of
measuring one GPU.  CPU only: the ranks rendezvous over gloo and stop after
the checks (--dry-run)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, 'bench.py')


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'):
        e.pop(k, None)
    e.update(env or {})
    e['HIP_VISIBLE_DEVICES'] = e.get('HIP_VISIBLE_DEVICES', '')
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, cwd=REPO, env=e)


def _line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_gpus2_starts_two_ranks_gloo():
    r = _run(['--gpus', '2', '--dist-backend', 'gloo', '--dry-run'])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d['dry_run'] is True
    assert d['rccl_world'] == 2 and d['dist_backend'] == 'gloo'
    assert len(d['rank_devices']) == 2
    # n_gpus counts distinct cards (none here: gloo ranks on the CPU)
    assert d['n_gpus'] == len({x for x in d['rank_devices'] if x >= 0})


def test_gpus3_starts_three_ranks_gloo():
    r = _run(['--gpus', '3', '--dist-backend', 'gloo', '--dry-run'])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d['rccl_world'] == 3 and len(d['rank_devices']) == 3
    assert d['n_gpus'] == len({x for x in d['rank_devices'] if x >= 0})


def test_gpus2_without_enough_gpus_is_refused():
    # RCCL (the default backend) needs a GPU per rank: this container has none,
    # as a one-GPU box has fewer than two
    r = _run(['--gpus', '2', '--dry-run'], env={'HIP_VISIBLE_DEVICES': ''})
    assert r.returncode != 0
    assert 'needs 2 GPUs' in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith('{')]


def test_world_size_must_match_gpus():
    # a torchrun environment of one rank while --gpus asks for two
    r = _run(['--gpus', '2', '--dry-run'], env={'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode != 0
    assert '--gpus 2' in r.stderr


def test_gpus1_is_one_process():
    r = _run(['--gpus', '1', '--dry-run'])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d['n_gpus'] == 1 and d['rccl_world'] == 1 and d['dist_backend'] is None
