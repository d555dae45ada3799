"""bench.py -- TPE suggestion-round throughput on MI355X.

Workload (BASELINE.json configs[2], the metric's "10k-trial history"):
32 hyperparameters, kind = i mod 5 in {uniform(-5,5), loguniform(-5,2),
quniform(0,100,1), normal(0,3), choice(5)}, N = 10000 synthetic trials,
2^24 EI candidates per label.

One step (default --mode fresh) = one suggestion of fmin's loop: append a
trial to the device-resident history, rebuild the posterior on the device
(numpy's tie order where it matters), build its expansion index, and run the
fused round -- Philox sampling of every label's candidates from l(x), lpdf
under l and g, broadcast_best maxloc per label -- then (N > 1) the winner
all-gather over RCCL.  Inputs are resident in HBM before the timed region.

N > 1 (torchrun, one rank per GPU): label shards by default -- rank r holds
the labels of parallel.label_shards(labels, N), their history columns,
posterior, index and whole rounds, each label keeping its Philox stream, so
the winners do not depend on N; --shard candidates splits every label's
candidates instead (rank r scores [r C/N, (r+1) C/N)).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision f64|f32]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Roofline of the dominant kernel (VALU-bound: neither HBM nor MFMA applies,
# DESIGN.md "Roofline").  `achieved` counts ALGORITHMIC work, SURVEY.md 8(d):
# per (candidate, component) eval d = x - mu, z = d s, t = fma(-z, z, c),
# e = exp(t), acc += e = 5 FLOP + 1 exp, quoted as 6 FLOP/eval, against the
# vendor vector peak for the dtype.
FLOPS_PER_EVAL = {'f64': 6.0, 'f32': 6.0}
# expansion screen (k_screen_bx): per candidate a 15-coefficient Horner
# polynomial (15 FMA) and the degree-5 exp(-kappa delta^2) factor (5 FMA)
BX_FLOPS_PER_CAND = 2 * 15 + 2 * 5
# The mark kernel k_hot_bx (round 6: the inverse-CDF draw, every candidate
# decided from its Philox words and a u-cell bit), algorithmic 32-bit lane operations per
# candidate: half a Philox4x32-10 call -- 10 rounds of two 32x32 -> 64-bit
# products (2 operations each: the low and high words) and two 3-input
# xors (2 each), 80 per call -- 40; the component pick (the guide's lookup
# and up to 3 threshold comparisons) 4; the u-cell bit (index, load, test)
# 3.  The fp64 draw of the ~0.8 % marked candidates and their sub-bin test
# run in k_hot_draw (not counted here).  Against the 32-bit VALU lane rate of MI355X_MICROARCH.md's
# vector figure (256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz = 78.6 T/s).
DRAW_OPS_PER_CAND = 47
PEAK_INT32_VECTOR_TOPS = 78.6
# Vector peaks.  FP32 157.3 TFLOP/s is MI355X_MICROARCH.md's figure (256 CUs
# x 4 SIMD-32 x 32 lanes x 2 FLOP x 2.4 GHz).  The guide lists no FP64
# figure: 78.6 TFLOP/s is AMD's MI355X specification for vector FP64 -- half
# the FP32 rate, which tools/ubench_issue.hip confirms on the box: a wave64
# v_fma_f64 issues in 4 cycles per SIMD against v_fma_f32's 2
# (profiles/r5b_issue_costs.json).
PEAK_FP64_VECTOR_TFLOPS = 78.6
PEAK_FP32_VECTOR_TFLOPS = 157.3
DENSE = ('dense', 'dense_lgmm1')   # 'dense': GMM1 + LGMM1 labels in one launch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--precision', default='f64', choices=['f64', 'f32'])
    ap.add_argument('--config', type=int, default=3, choices=[2, 3, 4, 5],
                    help='BASELINE.json config: 3 (headline, default), 2 (Hartmann-6, 2k '
                         'history, 2^20 candidates), 4 (nested SVM/RF/GBM choice space, 5k '
                         'history, 2^20 candidates), 5 (128 labels, 50k history, batched '
                         'new_ids x 24 candidates)')
    ap.add_argument('--agreement-steps', type=int, default=3,
                    help='f32: steps whose winners are compared with the exact fp64 round')
    ap.add_argument('--new-ids', type=int, default=4096,
                    help='config 5: new_ids per step in total, split over the ranks')
    ap.add_argument('--c5-history', type=int, default=50000,
                    help='config 5 history size (50000 = BASELINE.json; smaller only for experiments)')
    ap.add_argument('--labels', type=int, default=32)
    ap.add_argument('--trials', type=int, default=10000)
    ap.add_argument('--cand-log2', type=int, default=24,
                    help='log2 of the EI candidates per label in total (split over the ranks)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sample', type=int, default=2048,
                    help='candidates per label in the single-core numpy baseline sample')
    ap.add_argument('--cpu-sample-c', type=int, default=49152,
                    help='candidates per label in the all-cores C baseline sample')
    ap.add_argument('--no-latency', action='store_true')
    ap.add_argument('--no-projection', action='store_true',
                    help='skip the one-GPU projection of the 8-GPU step (profiling runs)')
    ap.add_argument('--no-screen', action='store_true',
                    help='f64: plain fp64 rounds (no fp32 screen); the winners are the same')
    ap.add_argument('--no-window', action='store_true',
                    help='f64: the plain fp32 screen (every term) instead of the windowed one')
    ap.add_argument('--win-t', type=int, default=16,
                    help='the windowed screen\'s cut T (components left out stay below 2^-T)')
    ap.add_argument('--win-groups', type=int, default=0,
                    help='label groups of a windowed round sorted on a second stream (0 = auto)')
    ap.add_argument('--unscreened-steps', type=int, default=4,
                    help='f64: plain fp64 rounds on the seeds of screened rounds, compared bit '
                         'for bit (screened_equals_fp64; 0 = skip)')
    ap.add_argument('--mode', default='fresh', choices=['fresh', 'warm'],
                    help='fresh (default): every step appends a trial and rebuilds the posterior '
                         'and its index, as fmin does; warm: rounds on one resident posterior')
    ap.add_argument('--append', type=int, default=1,
                    help='fresh mode: trials appended to the history per step')
    ap.add_argument('--devices', default=None,
                    help='one process, one multi-device context over these HIP ordinals '
                         '(e.g. 0,1,2,3; tpe_ctx_create_multi): the 1..8-GPU curve without '
                         'torchrun; a repeated ordinal shares that GPU (tests)')
    ap.add_argument('--shard', default='auto', choices=['auto', 'labels', 'candidates', 'descriptors'],
                    help='N > 1: label shards (each rank holds a subset of the labels: their '
                         'history, posterior, index and whole rounds; auto when every rank gets at '
                         'least one label), candidate shards (every label, C/N candidates each) or '
                         'descriptors (label shards build the posteriors and index, one all-gather '
                         'shares them, candidate shards score: parallel.DescriptorExchange)')
    ap.add_argument('--bx-split', type=int, default=None,
                    help='TPE_OPT_BX_SPLIT: workgroups per 64-bin block of the index tables (0 = auto)')
    ap.add_argument('--no-defer-report', action='store_true',
                    help='the quantized labels\' subset rebuild waits for its report before the round '
                         '(posterior.DEFER_REPORT off)')
    ap.add_argument('--bx-t', type=int, default=None,
                    help='TPE_OPT_BX_T: the expansion index\'s window cut T (0 = auto: 64 for tile rounds)')
    ap.add_argument('--dist-backend', default='nccl',
                    help='nccl (RCCL over xGMI); gloo only to rehearse N ranks on one GPU')
    ap.add_argument('--no-agreement', action='store_true',
                    help='skip the oracle leg: argmax agreement with the numpy restatement of the '
                         'reference on the near-ties of one round (oracle/near_ties.py)')
    ap.add_argument('--value-only', type=int, default=None,
                    help='1/0: TPE_OPT_VALUE_ONLY (default: on, as tpe.suggest, except for '
                         'candidate shards)')
    ap.add_argument('--aux-families', type=int, default=None,
                    help='1/0: the quantized and categorical labels on the second stream during sampled rounds '
                         '(TPE_OPT_AUX_FAMILIES; default: on, as tpe.suggest runs them, except candidate shards)')
    ap.add_argument('--early-orders', type=int, default=None,
                    help='1/0: the known labels\' argsorts under the first build '
                         '(posterior.EARLY_ORDERS)')
    ap.add_argument('--overlap-min-dense', type=int, default=None,
                    help='dense labels from which a fresh step builds order-free first and runs the '
                         'index beside the tie orders (workloads.OVERLAP_MIN_DENSE)')
    ap.add_argument('--sort-threads', type=int, default=None,
                    help='threads of the tie-order argsort pool (posterior.SORT_THREADS)')
    ap.add_argument('--no-other-configs', action='store_true',
                    help='config 3 at N=1: skip the legs of configs 2, 4 and 5 (child processes)')
    ap.add_argument('--dry-run', action='store_true',
                    help='launch and check the N ranks (rendezvous, world size, devices) and print '
                         'a {"dry_run": ...} line instead of measuring (CPU tests of the launcher)')
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N > 1` without a torchrun environment: start N rank processes
    of this script under torch.distributed.run (one per GPU, rendezvous on
    127.0.0.1) and return their exit code.  Runs before this process touches
    the GPU: torch.cuda.device_count() does not initialise HIP on this image,
    so the check below is safe, and the ranks are children, not an exec."""
    import subprocess
    if args.dist_backend == 'nccl':
        import torch
        n_dev = torch.cuda.device_count()
        if n_dev < args.gpus:
            sys.stderr.write('bench.py: --gpus %d needs %d GPUs, this node has %d: refusing to run %d '
                             'ranks on fewer devices (use --dist-backend gloo for a rehearsal on a '
                             'shared GPU)\n' % (args.gpus, args.gpus, n_dev, args.gpus))
            return 3
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault('OMP_NUM_THREADS', '4')
    return subprocess.call(cmd, env=env, cwd=REPO)


def distinct_gpus(rank_devices):
    """The GPUs the ranks ran on, each counted once (a rank without one:
    device -1, the CPU dry runs)."""
    return len({d for d in rank_devices if d is not None and d >= 0})


def check_world(args, dist, torch):
    """Every rank: the process group is the N ranks --gpus asked for, and
    under RCCL each rank has a GPU of its own.  Returns the per-rank device
    ordinals (all-gathered) or exits non-zero."""
    world = dist.get_world_size()
    if world != args.gpus:
        sys.stderr.write('bench.py: --gpus %d but the process group has %d ranks\n' % (args.gpus, world))
        sys.exit(3)
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))
    n_dev = torch.cuda.device_count()
    if args.dist_backend == 'nccl' and n_dev < local_world:
        sys.stderr.write('bench.py: %d ranks on this node but %d GPUs: RCCL needs one GPU per rank\n'
                         % (local_world, n_dev))
        sys.exit(3)
    dev = int(os.environ.get('LOCAL_RANK', '0')) % max(n_dev, 1) if n_dev else -1
    devs = [None] * world
    dist.all_gather_object(devs, dev)
    return devs


def other_configs(args):
    """BASELINE configs 2, 4 and 5 on the same box, each its own bench.py
    child process (started before this process touches the GPU; default
    steps): fresh step, warm round, screened_equals_fp64 and the one-GPU
    projection of the 8-GPU step from each child's own line."""
    import subprocess
    out = {}
    for cfg in (2, 4, 5):
        cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--config', str(cfg), '--steps',
               str(args.steps), '--warmup', str(args.warmup), '--no-cpu-baseline', '--no-latency']
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
        except subprocess.TimeoutExpired:
            out['config%d' % cfg] = {'error': 'timed out after 300 s'}
            continue
        wall = time.perf_counter() - t0
        lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
        if r.returncode != 0 or not lines:
            out['config%d' % cfg] = {'error': 'rc %d' % r.returncode, 'stderr_tail': r.stderr[-400:]}
            continue
        d = json.loads(lines[-1])
        st, pr = d.get('step') or {}, d.get('scaling_projection') or {}
        dp = d.get('scaling_projection_descriptors') or {}
        ag = d.get('oracle_near_tie_agree') or d.get('oracle_batched_agree')
        out['config%d' % cfg] = {
            'workload': d['config']['workload'], 'value': d['value'], 'unit': d['unit'],
            'fresh_step_ms': round(d['ms_per_step'], 3), 'warm_round_ms': st.get('warm_round_ms'),
            'expansion_index_ms': st.get('expansion_index_ms'),
            'screened_equals_fp64': d.get('screened_equals_fp64'),
            'projected_8gpu_efficiency_fresh': pr.get('projected_8gpu_efficiency_fresh'),
            'projected_8gpu_efficiency_warm': pr.get('projected_8gpu_efficiency_warm'),
            'projection_partition': pr.get('partition'),
            'projected_8gpu_efficiency_fresh_descriptors': dp.get('projected_8gpu_efficiency_fresh'),
            'projected_8gpu_efficiency_warm_descriptors': dp.get('projected_8gpu_efficiency_warm'),
            'rescored_per_step': (d.get('screen') or {}).get('rescored_per_step'),
            'oracle_agree': {k: ag.get(k) for k in ('cells', 'agree', 'rate')} if ag else None,
            'child_wall_s': round(wall, 1)}
    return out


def cpu_baseline_numpy(posts, n_cand):
    """The numpy restatement of the reference (oracle/tpe_oracle.py, test
    infra) on ONE host core: sample + score + argmax for every label."""
    from oracle import tpe_oracle as O
    rng = np.random.RandomState(1)
    evals = 0
    t0 = time.perf_counter()
    for p in posts:
        if p.family == 'categorical':
            cand = rng.multinomial(1, p.below, size=n_cand).argmax(1)
            lb, la = O.categorical_lpdf(cand, p.below), O.categorical_lpdf(cand, p.above)
            evals += 2 * n_cand
        else:
            samp = O.gmm1_sample if p.family == 'GMM1' else O.lgmm1_sample
            f = O.gmm1_lpdf if p.family == 'GMM1' else O.lgmm1_lpdf
            cand = samp(*p.below, low=p.low, high=p.high, q=p.q, rng=rng, size=(n_cand,))
            lb = f(cand, *p.below, low=p.low, high=p.high, q=p.q)
            la = f(cand, *p.above, low=p.low, high=p.high, q=p.q)
            evals += n_cand * (len(p.below[0]) + len(p.above[0]))
        O.broadcast_best_index(lb, la)
    dt = time.perf_counter() - t0
    return evals / dt, dt, evals


def cpu_baseline_c(eng, posts, n_cand, seed, rnd):
    """The C restatement of the reference's scoring (oracle/tpe_score.c, test
    infra, OpenMP over candidates on all the threads OMP gives it): the first
    n_cand candidates of every label's GPU candidate set (re-drawn through the
    engine's sampler entry points, untimed) scored under l and g + argmax."""
    from oracle import c_oracle as C
    cands = []
    for li, p in enumerate(posts):
        if p.family == 'categorical':
            cands.append(eng.categorical(p.below, seed=seed, size=(n_cand,), stream=li, round=rnd))
        else:
            samp = eng.GMM1 if p.family == 'GMM1' else eng.LGMM1
            cands.append(samp(*p.below, low=p.low, high=p.high, q=p.q, seed=seed,
                              size=(n_cand,), stream=li, round=rnd))
    evals = 0
    t0 = time.perf_counter()
    for p, cand in zip(posts, cands):
        if p.family == 'categorical':
            lb, la = C.categorical_lpdf(cand, p.below), C.categorical_lpdf(cand, p.above)
            evals += 2 * n_cand
        else:
            f = C.gmm1_lpdf if p.family == 'GMM1' else C.lgmm1_lpdf
            lb = f(cand, *p.below, low=p.low, high=p.high, q=p.q)
            la = f(cand, *p.above, low=p.low, high=p.high, q=p.q)
            evals += n_cand * (len(p.below[0]) + len(p.above[0]))
        C.broadcast_best_index(lb, la)
    dt = time.perf_counter() - t0
    return evals / dt, dt, evals, C.threads()


def near_tie_leg(eng, hist_full, res, seed, rnd, C):
    """Oracle leg (test infra, untimed): the round `res` (a warm step on the
    last fresh posterior) against the numpy restatement of the reference --
    per label numpy's broadcast_best argmax over the round's candidates (the
    64 best by HIP fp64 score re-scored in numpy for dense labels, every
    distinct value for quantized and categorical ones) must be the winner."""
    from oracle import near_ties as NT
    t0 = time.perf_counter()
    posts = NT.posteriors_of(eng, hist_full.labels)
    cells = NT.round_agreement(eng, posts, res, seed, rnd, C)
    d = NT.summary(cells)
    d.update({'round': rnd, 'seed': seed, 'wall_s': round(time.perf_counter() - t0, 1),
              'note': 'per (round, label) cell: the winner equals numpy\'s argmax (oracle/near_ties.py); '
                      'numpy_top2_gap = numpy\'s own best-minus-second score among the near-ties, '
                      'max_abs_hip_minus_numpy = the largest |HIP fp64 - numpy| score difference seen'})
    return d


def batched_oracle_leg(eng, hist_full, res, seed, ids, C, n_rows=8):
    """Config 5's oracle leg (test infra, untimed): n_rows random rounds of
    the first warm step x every label, the 24 candidates re-drawn and scored
    by the C restatement of the reference (oracle/tpe_score.c) -- numpy's
    broadcast_best argmax must be the round's index and value
    (oracle/near_ties.batched_agreement)."""
    from oracle import near_ties as NT
    t0 = time.perf_counter()
    posts = NT.posteriors_of(eng, hist_full.labels)
    rows = np.random.RandomState(11).choice(len(ids), min(n_rows, len(ids)), replace=False)
    cells = NT.batched_agreement(eng, posts, res, seed, ids, C, rows)
    agree = sum(c['agree'] for c in cells)
    return {'cells': len(cells), 'agree': agree, 'rate': agree / max(len(cells), 1),
            'rows': [int(r) for r in rows], 'wall_s': round(time.perf_counter() - t0, 1),
            'note': 'config 5: %d random rounds of the first warm step x all labels; per cell the 24 '
                    'candidates re-drawn and scored by oracle/tpe_score.c (the C restatement of '
                    'tpe.py:110-172, 265-307, 56-63), broadcast_best argmax (tpe.py:769-778) vs the '
                    'round\'s index and value' % len(rows)}


def config1_fmin(n_reps=3):
    """BASELINE config 1 on the HIP path: fmin((x - 3)^2, hp.uniform('x', -5,
    5), tpe.suggest, max_evals=100, rstate=RandomState(0)) -- the reference's
    test_fmin.py:24-35 -- wall seconds (median of n_reps, the engine warm),
    beside the reference's 0.141 s on one CPU core."""
    import hyperopt_amd as H
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.engine import get_engine
    get_engine(0, 'f64')
    walls, best = [], None
    for _ in range(n_reps):
        t0 = time.perf_counter()
        best = H.fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5), algo=tpe.suggest, max_evals=100,
                      trials=H.Trials(), rstate=np.random.RandomState(0))
        walls.append(time.perf_counter() - t0)
    return float(np.median(walls)), best['x']


def suggest_latency(n_labels, n_trials, n_reps=20, n_warm=3):
    """End-to-end tpe.suggest wall time (history gather + posterior build +
    H2D + fused GPU round + D2H + trial doc) at the reference defaults
    (n_EI_candidates=24), median of n_reps after n_warm warm-ups."""
    from hyperopt_amd import tpe
    from hyperopt_amd.base import Domain
    from hyperopt_amd.workloads import history_trials, hp_space, mixed_history
    hist = mixed_history(n_labels, n_trials, seed=0)
    trials = history_trials(hist)
    domain = Domain(lambda d: 0.0, hp_space(hist.labels))
    times = []
    for i in range(n_warm + n_reps):
        t0 = time.perf_counter()
        tpe.suggest([n_trials + i], domain, trials, 1000 + i)
        times.append(time.perf_counter() - t0)
    return float(np.median(times[n_warm:])) * 1e3


PMC_MIN_CLOCK_GHZ = 2.0


def measured_pmc(kernel_prefix, summary_glob='r*_pmc_summary.json'):
    """The dominant kernel's counters from the newest committed PMC summary
    that has it (rocprofv3 --pmc passes of this bench, tools/prof_round.sh +
    tools/pmc_summary.py): {} if absent; {'source': ... refused} when the
    counter run held a clock below 2 GHz.  Keys: hbm_bytes (2 x FETCH_SIZE +
    WRITE_SIZE per launch, the gfx950 correction), valu_busy (rocprofv3
    VALUBusy), issue_frac (the cycle-weighted issue model: per instruction
    class its count x the issue cost tools/ubench_issue.hip measured, over the
    launch's SIMD cycles), wave_cycles (where the waves' cycles go),
    instructions per candidate / eval, the counter run's clock."""
    import glob
    import re

    def tag_key(f):   # r<round><letters>: by round, then r2z < r2aa < r2ai (newest last)
        m = re.match(r'r(\d+)([a-z]*)_', os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, '')
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', summary_glob)), key=tag_key)
    for f in reversed(files):
        d = json.load(open(f))
        for name, v in d.items():
            if name.startswith(kernel_prefix) and '_hbm_bytes_per_launch' in v:
                # a counter run well below the bench's clock says little
                # about the timed kernel: refuse it
                clk = v.get('_eff_clock_ghz')
                src = os.path.relpath(f, REPO)
                if clk is None or clk < PMC_MIN_CLOCK_GHZ:
                    return {'source': '%s refused: effective clock %s GHz < %.1f' % (
                        src, 'unrecorded' if clk is None else '%.2f' % clk, PMC_MIN_CLOCK_GHZ)}
                out = {'source': '%s (%.2f GHz)' % (src, clk), 'kernel': name,
                       'hbm_bytes': v['_hbm_bytes_per_launch'], 'valu_busy': v.get('_valu_busy'),
                       'issue_frac': v.get('_issue_frac'), 'issue_split': v.get('_issue_split'),
                       'issue_costs': v.get('_issue_costs_source'),
                       'wave_cycles': v.get('_wave_cycle_split'),
                       'instr_per_candidate': v.get('_valu_instr_per_candidate'),
                       'instr_per_eval': v.get('_valu_instr_per_eval'), 'clock_ghz': clk}
                return {k: x for k, x in out.items() if x is not None}
    return {}


def descriptor_projection(args, hist_full, dev, screen, value_only, C_total, p0, full_fresh_ms, full_warm_ms):
    """One GPU running each rank's share of the descriptor-exchange step
    (parallel.DescriptorExchange) in turn: max over shards of (append +
    rebuild + index + export) + the import of all 8 blobs + one rank's slice
    of the round (the slices cost alike: whole_n / whole_rounds keep the
    whole round's size choices).  The two all-gathers are not run (one GPU):
    the blobs' bytes are reported with a ring estimate beside."""
    import torch
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.parallel import _align, label_shards
    from hyperopt_amd.workloads import FminLoop
    world = 8
    c5 = args.config == 5
    rounds_total = args.new_ids if c5 else 1
    shards = label_shards(hist_full.labels, world)

    def opts(e):
        for k, v in (('screen', int(screen)), ('window', int(not args.no_window)), ('win_t', args.win_t),
                     ('win_groups', args.win_groups),
                     ('value_only', value_only if c5 else 0), ('aux_families', 1 if c5 else 0)):
            e.set_option(k, v)

    engs, loops, blobs = [], [], []
    per = []
    try:
        for sh in shards:
            e = Engine(dev, args.precision)
            engs.append(e)
            opts(e)
            lp = FminLoop(hist_full, label_ids=sh)
            lp.advance(e, args.trials + (p0 - 1) * args.append)
            loops.append(lp)
            blobs.append(None)

        def build(k, pos):
            loops[k].advance(engs[k], args.trials + pos * args.append, n_candidates=C_total,
                             n_rounds=rounds_total)
            n = engs[k].export_size()
            if blobs[k] is None or blobs[k].numel() < n:
                blobs[k] = torch.empty(_align(n) + (1 << 20), dtype=torch.uint8, device='cuda')
            return engs[k].export_posterior(blobs[k])

        sizes = [0] * world
        for k in range(world):
            for w in (p0, p0 + 1):
                build(k, w)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                sizes[k] = build(k, p0 + 2 + i)
            torch.cuda.synchronize()
            per.append((time.perf_counter() - t0) / args.steps * 1e3)
        slot = _align(max(sizes))
        allb = torch.empty(world * slot, dtype=torch.uint8, device='cuda')
        for k in range(world):
            allb[k * slot:k * slot + sizes[k]] = blobs[k][:sizes[k]]
        for e in engs:
            e.close()
        engs = []
        imp = Engine(dev, args.precision)
        engs.append(imp)
        opts(imp)
        offs = [k * slot for k in range(world)]
        imp.import_posterior(allb, offs, shards)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            imp.import_posterior(allb, offs, shards)
        torch.cuda.synchronize()
        t_imp = (time.perf_counter() - t0) / args.steps * 1e3
        if c5:
            imp.set_option('whole_rounds', args.new_ids)
            nloc = args.new_ids // world

            def rnd(i):
                return imp.suggest_batch(1234, list(range(i * args.new_ids, i * args.new_ids + nloc)), C_total)
        else:
            imp.set_option('whole_n', C_total)

            def rnd(i):
                return imp.suggest(1234 + i, C_total // world, round=i, cand_offset=0)
        # (a fresh import: the first round builds the per-posterior caches
        # the fresh step pays -- timed as such; the warm slice after it)
        t_first = []
        t_warm = []
        for i in range(args.steps + 1):
            imp.import_posterior(allb, offs, shards)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rnd(p0 + i)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rnd(p0 + i)
            torch.cuda.synchronize()
            if i:
                t_first.append((t1 - t0) * 1e3)
                t_warm.append((time.perf_counter() - t1) * 1e3)
        t_first, t_warm = float(np.mean(t_first)), float(np.mean(t_warm))
    finally:
        for e in engs:
            e.close()
    # ring all-gather of the blobs over xGMI: 7 hops of one slot at ~64 GB/s
    # achieved per link (MI355X_MICROARCH.md: 153 GB/s peak) + ~10 us a hop
    gather_ms = 7 * (slot / 64e9 * 1e3 + 0.010)
    fresh = max(per) + t_imp + t_first
    return {'partition': 'descriptor exchange (label shards build, one all-gather of the posteriors, '
                         '%s)' % ('new_id shards' if c5 else 'candidate shards, C/8 per label'),
            'labels_per_shard': [len(sh) for sh in shards],
            'build_export_ms_per_shard': [round(x, 3) for x in per],
            'import_ms': round(t_imp, 3), 'slice_round_first_ms': round(t_first, 3),
            'slice_round_warm_ms': round(t_warm, 3),
            'blob_bytes_per_shard': sizes, 'allgather_estimate_ms': round(gather_ms, 3),
            'fresh_step_ms_shard': round(fresh, 3), 'warm_round_ms_shard': round(t_warm, 3),
            'projected_8gpu_efficiency_fresh': full_fresh_ms / (8.0 * fresh),
            'projected_8gpu_efficiency_fresh_with_gather_estimate': full_fresh_ms / (8.0 * (fresh + gather_ms)),
            'projected_8gpu_efficiency_warm': full_warm_ms / (8.0 * t_warm),
            'note': 'one GPU running each rank\'s share in turn: T(whole) / (8 T(rank)), T(rank) = '
                    'max_r(build_r + export_r) + import + the first slice round on the imported posterior '
                    '(warm: the slice round); the all-gathers are estimated, not run -- a projection'}


def roofline_lpdf(launch_ms, evals, args):
    """The lpdf kernel north_star's target describes:
    the plain fp64 round k_round<double> (GMM1_lpdf / LGMM1_lpdf of every
    (candidate, component) pair, tpe.py:110-172, logsum_rows :259-262), timed
    by HIP events on the engine's stream in this run's unscreened leg, with
    the counters of its committed PMC passes (tools/gpu.sh lpdf ->
    profiles/r*_lpdf_pmc_summary.json)."""
    pmc = (measured_pmc('k_round<double, 8, true', 'r*_lpdf_pmc_summary.json')
           if args.config == 3 and args.cand_log2 == 24 and args.labels == 32 else {})
    rate = evals / (launch_ms * 1e-3)
    achieved = rate * FLOPS_PER_EVAL['f64'] / 1e12
    issue = pmc.get('issue_frac')
    return {'kernel': 'k_round<double, DENSE_ANY, SAMPLE> (plain fp64 round: Philox draw, GMM1/LGMM1 lpdf '
                      'under l and g of every (candidate, component) pair, block maxloc)',
            'evals_per_launch': evals, 'launch_ms': round(launch_ms, 3), 'evals_per_s': rate,
            'target_evals_per_s': 1e11, 'meets_rate_target': rate >= 1e11,
            'achieved': round(achieved, 3), 'peak': PEAK_FP64_VECTOR_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(achieved / PEAK_FP64_VECTOR_TFLOPS, 4), 'flops_per_eval': FLOPS_PER_EVAL['f64'],
            'valu_instr_per_eval': pmc.get('instr_per_eval'), 'issue_frac_measured': issue,
            'issue_split': pmc.get('issue_split'), 'valu_busy_measured': pmc.get('valu_busy'),
            'wave_cycles': pmc.get('wave_cycles'), 'pmc_source': pmc.get('source'),
            'meets_50pct_valu_roofline': (issue >= 0.5) if issue is not None else None,
            'note': 'north_star: >= 1e11 lpdf evals/s at >= 50 % of the VALU roofline.  The VALU roofline '
                    'here is the cycle-weighted issue rate (issue_frac_measured: PMC instruction classes '
                    'x the issue costs tools/ubench_issue.hip measured); frac counts only the 6 '
                    'algorithmic FLOP of an eval against the fp64 vector peak -- the fp64 exp costs ~7 '
                    'instructions beyond them (an LDS-table + degree-3 polynomial sequence), so the '
                    'kernel is issue-bound well below that FLOP peak'}


def workload_name(args, C):
    if args.config == 2:
        return 'config2: Hartmann-6 over hp.uniform, N=2000 history, 2^20 EI candidates ' \
               'per label (C/N per GPU)'
    if args.config == 4:
        return 'config4: nested hp.choice SVM/RF/GBM space (13 labels), N=5000 history, ' \
               '2^%d EI candidates per label (C/N per GPU)' % args.cand_log2
    if args.config == 5:
        return 'config5: 128-dim mixed space, N=%d history, %d new_ids per step x 24 EI ' \
               'candidates (labels or new_ids split over the GPUs, winners all-gathered)' % (
                   args.trials, args.new_ids)
    return 'config3: %d-dim mixed space, N=%d history, 2^%d EI candidates per label ' \
           '(labels split over the GPUs)' % (args.labels, args.trials, args.cand_log2)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit('--gpus must be >= 1')
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1 and not args.devices:
        sys.exit(launch_ranks(args))   # N rank processes under torch.distributed.run
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != (1 if args.devices else args.gpus):
        sys.stderr.write('bench.py: WORLD_SIZE=%d but --gpus %d%s\n' % (
            world, args.gpus, ' (--devices runs one process)' if args.devices else ''))
        sys.exit(3)
    others = None
    if (world == 1 and args.config == 3 and not args.devices and not args.no_other_configs
            and args.precision == 'f64' and args.labels == 32 and args.cand_log2 == 24
            and not args.dry_run):
        others = other_configs(args)   # (child processes, before this one touches the GPU)
    import torch
    dist = None
    rank_devices = [local]
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == 'nccl' or torch.cuda.device_count():
            local = local % max(torch.cuda.device_count(), 1)
            if not args.dry_run:
                torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
        rank_devices = check_world(args, dist, torch)
    if args.dry_run:
        if dist is not None:
            dist.barrier()
        if rank == 0:
            print(json.dumps({'dry_run': True, 'n_gpus': distinct_gpus(rank_devices),
                              'rccl_world': world if dist else 1,
                              'dist_backend': args.dist_backend if dist else None,
                              'rank_devices': rank_devices}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    from hyperopt_amd import posterior as P
    if args.sort_threads is not None:
        P.SORT_THREADS = args.sort_threads
    if args.early_orders is not None:
        P.EARLY_ORDERS = bool(args.early_orders)
    if args.overlap_min_dense is not None:
        from hyperopt_amd import workloads as W
        W.OVERLAP_MIN_DENSE = args.overlap_min_dense
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import (FminLoop, conditional_history, hartmann_history,
                                         mixed_history)

    # the synthetic history holds the trials the fresh-posterior steps append
    # (fmin's loop: one trial per suggestion) after the first args.trials
    extra = (args.warmup + 4 * args.steps + 2) * args.append
    if args.config == 2:
        args.labels, args.trials, args.cand_log2 = 6, 2000, 20
        hist_full = hartmann_history(args.trials + extra, seed=0)
    elif args.config == 4:
        args.trials, args.cand_log2 = 5000, 20
        hist_full = conditional_history(args.trials + extra, seed=0)
        args.labels = len(hist_full.labels)
    elif args.config == 5:
        args.labels, args.trials = 128, args.c5_history
        hist_full = mixed_history(args.labels, args.trials + extra, seed=0)
    else:
        hist_full = mixed_history(args.labels, args.trials + extra, seed=0)
    hist = hist_full.prefix(args.trials)
    # the resident posterior: built on the device from the history (the
    # product path for histories this size, tpe.suggest posterior_builder
    # 'auto'); the host numpy build is timed beside it
    devs = [int(d) for d in args.devices.split(',')] if args.devices else None
    if devs and world > 1:
        raise SystemExit('--devices is the single-process multi-GPU mode; not under torchrun')
    eng = Engine(devs if devs else local, args.precision)
    t_host = time.perf_counter()
    posts = hist.posteriors()
    descs, w, m, s = P.pack(posts)
    t_host = time.perf_counter() - t_host
    inputs = hist.device_inputs()
    dev_call, dev_kern = [], []
    for _ in range(3):
        t0 = time.perf_counter()
        eng.build_posterior(*inputs, gamma=0.25, prior_weight=1.0)
        dev_call.append(time.perf_counter() - t0)
        dev_kern.append(eng.last_build_ms())
    post_build = {'device_call_ms': round(1e3 * float(np.median(dev_call)), 3),
                  'device_kernels_ms': round(float(np.median(dev_kern)), 3),
                  'host_numpy_ms': round(1e3 * t_host, 3),
                  'note': 'tpe_build_posterior (split, sort, Parzen, fold on the GPU; call '
                          'includes the H2D of the history) vs posterior.py + pack'}
    C_total = 24 if args.config == 5 else 1 << args.cand_log2
    from hyperopt_amd.parallel import gather_labels, label_shards
    # label shards whenever every rank gets a label (r4am: config 4's 13 labels
    # over 8 ranks project 0.25 / 0.28 against 0.14 / 0.15 as candidate shards)
    by_label = (args.shard == 'labels' or
                (args.shard == 'auto' and len(hist_full.labels) >= max(world, 8 if world == 1 else 1)))
    # descriptor exchange: this rank builds its label shard's posteriors and
    # index, every rank scores its candidate slice (config 5: its new_ids) of
    # every label on the shared posterior
    desc = args.shard == 'descriptors' and world > 1
    if desc:
        by_label = False
    shards = label_shards(hist_full.labels, world) if (by_label or desc) else None
    if desc:
        ids_local = args.new_ids // world
        C = C_total   # (the exchange slices every label's candidates: rank r's [r C/N, (r+1) C/N))
        if args.config == 5 and args.new_ids % world:
            raise SystemExit('--new-ids must divide over %d ranks' % world)
    elif by_label:   # whole rounds of this rank's labels
        ids_local, C = args.new_ids, C_total
    elif args.config == 5:
        if args.new_ids % world:
            raise SystemExit('--new-ids must divide over %d ranks' % world)
        ids_local, C = args.new_ids // world, C_total
    else:
        if C_total % world:
            raise SystemExit('2^%d candidates must divide over %d ranks' % (args.cand_log2, world))
        C = C_total // world
    L = len(posts)

    from hyperopt_amd.parallel import DescriptorExchange, DeviceExchange
    if desc:
        xch = DescriptorExchange(eng, shards, rank, split='rounds' if args.config == 5 else 'candidates')
    else:
        xch = (DeviceExchange(eng, 'labels' if by_label else ('rounds' if args.config == 5 else 'candidates'),
                              shards=shards, rank=rank) if dist is not None else None)

    # fresh-posterior steps (default): each step appends the next trial(s) to
    # the device-resident history and rebuilds the posterior as tpe.suggest
    # does (FminLoop), so the round pays the expansion index of a new
    # posterior -- what every suggestion of fmin's loop pays
    loop = None
    fresh_mode = args.mode == 'fresh'
    if fresh_mode or ((by_label or desc) and world > 1):
        loop = FminLoop(hist_full, label_ids=shards[rank] if (by_label or desc) and world > 1 else None)
        loop.advance(eng, args.trials)        # untimed: the initial history, uploaded whole
        if desc:
            xch.share()                       # (warm mode: the shared posterior of that history)
    results = {}

    def step(i, fresh, n=None, e=None, lp=None, gather=True):
        """One step; n: the candidates per label of this rank's candidate
        shard (default C) -- the candidate-shard projection runs one eighth
        of a round; e, lp: another engine and loop (the label-shard
        projection)."""
        e = eng if e is None else e
        lp = loop if lp is None else lp
        nc = C if n is None else n
        exchange = dist is not None and gather
        if desc:
            # this rank's labels rebuilt (their index queued for the whole
            # round's size), the posteriors shared, this rank's slice scored
            if fresh:
                t0 = time.perf_counter()
                lp.advance(e, args.trials + (i + 1) * args.append,
                           n_candidates=C_total if args.precision == 'f64' else 0,
                           n_rounds=args.new_ids if args.config == 5 else 1)
                xch.share()
                P._phase('step_total', t0)
            if args.config == 5:
                first_id = i * args.new_ids + rank * ids_local
                return xch.round(1234, list(range(first_id, first_id + ids_local)), C)
            return xch.round(1234 + i, [i], C)[0]
        off = 0 if by_label else rank * nc
        if args.config == 5:   # independent new_ids split over the GPUs (or each rank's labels)
            first_id = i * args.new_ids + (0 if by_label else rank * ids_local)
            ids = list(range(first_id, first_id + ids_local))
            if exchange:   # every rank ends with every new_id's winners
                def rnd():
                    return xch.round(1234, ids, C)
            else:
                def rnd():
                    return e.suggest_batch(seed=1234, rounds=ids, n_candidates=C)
        elif exchange:   # the winners (L x 48 B) all-gathered device to device
            def rnd():
                return xch.round(1234 + i, [i], nc, cand_offset=off)[0]
        else:
            def rnd():
                return e.suggest(seed=1234 + i, n_candidates=nc, round=i, cand_offset=off)
        if fresh:
            # the round runs inside advance as tpe.suggest runs it (the dense
            # labels' round under the host's tie-order argsorts), except
            # under the device exchange (its collective follows the round)
            t0 = time.perf_counter()
            out = lp.advance(e, args.trials + (i + 1) * args.append,
                             n_candidates=nc if args.precision == 'f64' else 0,
                             n_rounds=ids_local if args.config == 5 else 1,
                             round_call=None if exchange else rnd)
            P._phase('step_total', t0)
            if not exchange:
                return out[1]
        return rnd()

    def timed(n_steps, first, fresh, keep=False, n=None):
        """Run n_steps steps (barrier + sync on both sides); returns wall
        seconds (max over ranks) and the summed per-family / screen stats
        (scr[7]: the expansion-index wall ms of the steps that built one)."""
        mode_ms, mode_ev, scr = {}, {}, [0, 0, 0.0, 0, 0, 0, 0, 0.0]
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n_steps):
            res = step(first + i, fresh, n)
            if keep:
                results[first + i] = res
            for k, (ms, ev) in eng.last_mode_stats().items():
                mode_ms[k] = mode_ms.get(k, 0.0) + ms
                mode_ev[k] = mode_ev.get(k, 0) + ev
            a, b, ms = eng.last_screen(with_ms=True)
            scr[0] += a
            scr[1] += b
            scr[2] += ms
            scr[3] += eng.last_screen_terms()
            scr[4] += eng.last_rescore_terms()
            hl, hf = eng.last_hot()
            scr[5] += max(hl, 0)
            scr[6] += hf
            if fresh:
                scr[7] += eng.last_prepare_ms()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([dt], dtype=torch.float64,
                              device='cuda' if args.dist_backend == 'nccl' else 'cpu')
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        return dt, mode_ms, mode_ev, scr

    screen = args.precision == 'f64' and not args.no_screen
    eng.set_option('screen', int(screen))
    # value-only rounds as tpe.suggest runs them (engine.get_engine: the
    # winners' values are all a document needs, tpe.py:906-916) -- except
    # for candidate shards, whose winners merge by score (the packed map's
    # certified cells otherwise carry no fp64 lpdfs; tile rounds unchanged)
    value_only = (args.value_only if args.value_only is not None
                  else int(not (dist is not None and not by_label and args.config != 5)))
    eng.set_option('value_only', value_only)
    # the side families on the second stream, as tpe.suggest runs them
    # (engine.get_engine), except for candidate shards (as value_only)
    aux_families = (args.aux_families if args.aux_families is not None
                    else int(not (dist is not None and not by_label and args.config != 5)))
    eng.set_option('aux_families', aux_families)
    if args.bx_split is not None:
        eng.set_option('bx_split', args.bx_split)
    if args.no_defer_report:
        P.DEFER_REPORT = False
    if args.bx_t is not None:
        eng.set_option('bx_t', args.bx_t)
    eng.set_option('window', int(not args.no_window))
    eng.set_option('win_t', args.win_t)
    eng.set_option('win_groups', args.win_groups)
    if world > 1 and not by_label:   # one candidate shard: size choices follow the whole round
        eng.set_option('whole_rounds' if args.config == 5 else 'whole_n',
                       args.new_ids if args.config == 5 else C_total)
    for i in range(args.warmup):
        step(i, fresh_mode)
    # the expansion screen's index (bin tables, lists, sub-bin bounds) is
    # built once per posterior, in its first large round
    prep_ms = eng.last_prepare_ms() if args.warmup > 0 else None
    P.PHASES = {}     # host-timer breakdown of the timed steps' posterior work
    dt, mode_ms, mode_ev, scr = timed(args.steps, args.warmup, fresh_mode)
    phases, P.PHASES = P.PHASES, None
    smode_timed = eng.last_screen_mode()   # (the timed rounds' screen; later legs run others)
    # the same rounds on the posterior of the last step, reused (no append):
    # the round alone, and the reference for the unscreened comparison
    warm_first = args.warmup + args.steps
    wdt, _, _, _ = timed(args.steps, warm_first, False, keep=True) if fresh_mode else (None,) * 4
    # the plain fp64 round on the SAME (seed, round) as screened steps on
    # the same posterior -- before anything else advances it: winners,
    # values and lpdfs bit for bit
    unscreened = None
    if screen and args.unscreened_steps > 0 and world == 1 and devs is None:
        # (fresh mode compares the warm steps' rounds: at most args.steps of them)
        nu = min(args.unscreened_steps, args.steps) if fresh_mode else args.unscreened_steps
        first = warm_first if fresh_mode else args.warmup + args.steps
        if not fresh_mode:
            timed(nu, first, False, keep=True)
        eng.set_option('screen', 0)
        ures = {}
        u_ms = u_ev = 0.0   # the plain fp64 round's dense launch: device ms (HIP events), evals
        t0 = time.perf_counter()
        for i in range(nu):
            ures[first + i] = step(first + i, False)
            ms_ev = eng.last_mode_stats()
            u_ms += sum(ms_ev[k][0] for k in DENSE)
            u_ev += sum(ms_ev[k][1] for k in DENSE)
        torch.cuda.synchronize()
        udt = time.perf_counter() - t0
        eng.set_option('screen', 1)
        if value_only:   # index and value: the fields a value-only round reports for every cell
            same = all(np.array_equal(results[k]['index'], ures[k]['index']) and
                       results[k]['value'].tobytes() == ures[k]['value'].tobytes() for k in ures)
        else:
            same = all(results[k].view(np.uint8).tobytes() == ures[k].view(np.uint8).tobytes() for k in ures)
        unscreened = (same, udt, nu, first, u_ms, u_ev)
    # oracle leg (untimed): the first warm round against numpy's argmax, on
    # the posterior that produced it (before the projection advances it)
    agree_leg = None
    if (rank == 0 and world == 1 and devs is None and not args.no_agreement and fresh_mode
            and args.config in (2, 3, 4) and args.precision == 'f64' and warm_first in results):
        agree_leg = near_tie_leg(eng, hist_full, results[warm_first], 1234 + warm_first, warm_first, C)
    if (rank == 0 and world == 1 and devs is None and not args.no_agreement and fresh_mode
            and args.config == 5 and args.precision == 'f64' and warm_first in results):
        agree_leg = batched_oracle_leg(eng, hist_full, results[warm_first], 1234,
                                       list(range(warm_first * args.new_ids, warm_first * args.new_ids + ids_local)),
                                       C)
    # device memory after the timed steps: the library's buffers (their
    # high-water mark: they grow by 1/4 and are kept) and the whole device
    free_b, total_b = torch.cuda.mem_get_info()
    mem = {'library_bytes': eng.device_bytes(), 'device_used_bytes': int(total_b - free_b),
           'device_total_bytes': int(total_b),
           'note': 'library_bytes: tpe_device_bytes (posterior, resident history, expansion index, '
                   'hot lists, round buffers of this rank); device_used_bytes: hipMemGetInfo, '
                   'including the HIP / torch runtime'}
    # the 8-GPU step projected from this one GPU: each rank's share run
    # alone (label shards: an engine per shard holding its labels' history,
    # posterior and index, whole rounds, the slowest shard setting the step;
    # candidate shards: C/8 candidates per label at the whole round's map
    # choices, the per-posterior work repeated), fresh and warm
    proj = None
    if fresh_mode and world == 1 and devs is None and not args.no_projection and (by_label or (args.config != 5 and C % 8 == 0)):
        p0 = warm_first + args.steps
        if by_label:
            per = []
            for sh in label_shards(hist_full.labels, 8):
                e8 = Engine(local, args.precision)
                for k, v in (('screen', int(screen)), ('window', int(not args.no_window)),
                             ('win_t', args.win_t), ('win_groups', args.win_groups), ('value_only', value_only),
                             ('aux_families', aux_families)):
                    e8.set_option(k, v)
                l8 = FminLoop(hist_full, label_ids=sh)
                l8.advance(e8, args.trials + (p0 - 1) * args.append)
                for w in (p0 - 1, p0):                          # warm-up steps
                    step(w, True, e=e8, lp=l8, gather=False)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    step(p0 + 1 + i, True, e=e8, lp=l8, gather=False)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for i in range(args.steps):
                    step(p0 + 1 + i, False, e=e8, lp=l8, gather=False)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                per.append((len(sh), (t1 - t0) / args.steps * 1e3, (t2 - t1) / args.steps * 1e3))
                e8.close()
            pf, pw = max(x[1] for x in per), max(x[2] for x in per)
            proj = {'partition': 'label shards (parallel.label_shards, 8 ranks)',
                    'labels_per_shard': [x[0] for x in per],
                    'fresh_step_ms_per_shard': [round(x[1], 3) for x in per],
                    'warm_round_ms_per_shard': [round(x[2], 3) for x in per]}
        else:
            eng.set_option('whole_n', C)
            pf = timed(args.steps, p0, True, n=C // 8)[0] / args.steps * 1e3
            pw = timed(args.steps, p0 + args.steps, False, n=C // 8)[0] / args.steps * 1e3
            eng.set_option('whole_n', 0)
            proj = {'partition': 'candidate shards (C/8 per label)', 'shard_candidates_per_label': C // 8}
        proj.update({
            'fresh_step_ms_full': dt / args.steps * 1e3, 'fresh_step_ms_shard': pf,
            'warm_round_ms_full': wdt / args.steps * 1e3, 'warm_round_ms_shard': pw,
            'projected_8gpu_efficiency_fresh': dt / args.steps * 1e3 / (8.0 * pf),
            'projected_8gpu_efficiency_warm': wdt / args.steps * 1e3 / (8.0 * pw),
            'note': 'one GPU running each rank\'s share of the 8-GPU step in turn: efficiency = '
                    'T(whole) / (8 max_r T(shard r)); the RCCL all-gather of the winners (48 B per '
                    'label) is not in it -- a projection, not a measured scaling curve'})
    # the descriptor-exchange partition projected the same way: each rank's
    # fresh build of its label shard (history append, posterior, index) and
    # export, run shard by shard; one engine importing the 8 blobs, then its
    # slice of the round (C/8 candidates of every label; config 5: 1/8 of
    # the new_ids) -- the slowest build + import + slice
    dproj = None
    if (fresh_mode and world == 1 and devs is None and not args.no_projection and args.precision == 'f64'
            and args.shard in ('auto', 'descriptors') and (args.config == 5 or C % 8 == 0)
            and len(hist_full.labels) >= 8):
        dproj = descriptor_projection(args, hist_full, local, screen, value_only, C_total,
                                      warm_first + args.steps, dt / args.steps * 1e3,
                                      wdt / args.steps * 1e3)
    # `value` counts EXECUTED (candidate, component) lpdf terms (BASELINE.md
    # section 3): quantized labels their grid-table evals, screened dense
    # labels the fp32 terms the screen summed plus the fp64 terms of the
    # re-scored candidates; the reference-equivalent rate (every pair of
    # the round, as the reference's numpy evaluates them) is reported beside
    executed = sum(mode_ev.values())
    if scr[0] > 0:
        executed += scr[3] + scr[4] - sum(mode_ev.get(k, 0) for k in DENSE)
    executed_all = executed * world
    if dist is not None:   # the ranks' shards differ (label shards): sum what they executed
        te = torch.tensor([float(executed)], dtype=torch.float64,
                          device='cuda' if args.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(te)
        executed_all = int(te.item())
    value = executed_all / dt
    rounds_per_step = args.new_ids if args.config == 5 else 1
    ref_equiv_per_step = sum((2 if p.family == 'categorical' else len(p.below[0]) + len(p.above[0]))
                             * C_total * rounds_per_step for p in posts)

    # roofline of the dominant kernel (device time from HIP events on the
    # engine's stream, summed over the timed steps)
    prec = args.precision
    dom = max((k for k in mode_ms if k in DENSE), key=lambda k: mode_ms[k])
    screened = scr[0] > 0
    smode = smode_timed if screened else 0
    windowed = smode == 2
    hot = smode == 3 and scr[5] > 0
    if hot:
        # the hot-bin prefilter's mark kernel (k_hot_bx, the dominant
        # kernel; its HIP-event bracket holds it alone): every candidate's
        # Philox words, pick and u-cell bit; the marked ~0.8 % go to
        # k_hot_draw (fp64 draw + sub-bin bit, in other_dense_ms)
        dom_ms = scr[2]
        kprec = 'int32'
        kname = 'k_hot_bx<'
        kdesc = 'k_hot_bx (the hot-bin prefilter\'s mark kernel: every candidate\'s Philox4x32-10 words, ' \
                'component pick and u-cell bit; the marked ones go to k_hot_draw, which draws them by the ' \
                'inverse CDF in fp64 and lists those whose sub-bin can hold the winner), GMM1+LGMM1 labels'
        dom_rate = scr[3] / (dom_ms * 1e-3)
        dom_flops = scr[0] * DRAW_OPS_PER_CAND
    elif smode == 3:
        # the expansion screen: per candidate the below mixture and the
        # bin's list of unclipped components as direct fp64 terms (6 FLOP
        # each; tpe_last_screen_terms) and the bin's 13-term
        # polynomial + exp factor (BX_FLOPS_PER_CAND), over its device time
        dom_ms = scr[2]
        kprec = 'f64'
        kname = 'k_screen_bx<'
        kdesc = 'k_screen_bx (expansion screen of the fp64 round, GMM1+LGMM1 labels: below mixture ' \
                'and unclipped components as fp64 terms, the equal-sigma above components as a ' \
                'per-bin Taylor polynomial)'
        dom_rate = scr[3] / (dom_ms * 1e-3)
        dom_flops = scr[3] * FLOPS_PER_EVAL['f64'] + scr[0] * BX_FLOPS_PER_CAND
    elif screened:
        # the fp32 screening kernel: the (candidate, component) terms it
        # actually summed (tpe_last_screen_terms) over its own device time
        dom_ms = scr[2]
        kprec = 'f32'
        if windowed:
            kname, kdesc = 'k_screen_win<', 'k_screen_win (windowed fp32 screen of the fp64 ' \
                'round, GMM1+LGMM1 labels)'
        else:
            kname, kdesc = 'k_screen<', 'k_screen (fp32 screen of the fp64 round, GMM1+LGMM1 labels)'
        dom_rate = scr[3] / (dom_ms * 1e-3)
        dom_flops = scr[3] * FLOPS_PER_EVAL['f32']
    else:
        dom_ms = mode_ms[dom]
        kprec = prec
        kname = 'k_round<%s, %d, true,' % ('double' if prec == 'f64' else 'float',
                                           8 if dom == 'dense' else 1)
        kdesc = 'k_round<%s,%s>' % (prec, dom + ' (GMM1+LGMM1 labels)')
        dom_rate = mode_ev[dom] / (dom_ms * 1e-3)
        dom_flops = mode_ev[dom] * FLOPS_PER_EVAL[prec]
    peak = {'f64': PEAK_FP64_VECTOR_TFLOPS, 'f32': PEAK_FP32_VECTOR_TFLOPS,
            'int32': PEAK_INT32_VECTOR_TOPS}[kprec]
    # PMC figures come from the committed profile of the default workload
    # (config 3, tools/prof_round.sh): only that workload's line carries them
    pmc = (measured_pmc(kname) if args.config == 3 and world == 1 and args.cand_log2 == 24
           and args.labels == 32 else {})
    achieved = dom_flops / (dom_ms * 1e-3) / 1e12
    roof = {'bound': 'valu', 'kernel': kdesc,
            'achieved': round(achieved, 3), 'peak': peak, 'unit': 'Tops/s' if kprec == 'int32' else 'TFLOP/s',
            'frac': round(achieved / peak, 4), 'traffic': pmc.get('hbm_bytes'),
            'traffic_source': pmc.get('source'), 'valu_busy_measured': pmc.get('valu_busy'),
            'issue_frac_measured': pmc.get('issue_frac'), 'issue_split': pmc.get('issue_split'),
            'issue_costs_source': ('profiles/' + pmc['issue_costs']) if pmc.get('issue_costs') else None,
            'wave_cycles': pmc.get('wave_cycles'),
            'pmc_source': pmc.get('source'),
            'evals_per_s': dom_rate, 'flops_per_eval': FLOPS_PER_EVAL.get(kprec),
            'launch_ms': dom_ms / args.steps,
            'issue_model_note': 'issue_frac_measured: PMC instruction classes (SQ_INSTS_VALU_{ADD,MUL,FMA,'
                                'TRANS}_F64 / _F32, _INT32, _INT64, _CVT, the rest) x the cycles per wave64 '
                                'instruction per SIMD tools/ubench_issue.hip measured at 8 waves per SIMD '
                                '(SIMD-32: 2 for int32 / fp32, 4 for fp64 and v_mad_u64_u32, 8 for v_exp_f32, '
                                '16 for v_sqrt_f64), over 1024 SIMDs x the launch\'s cycles; valu_busy_measured: '
                                'rocprofv3 VALUBusy (SQ_ACTIVE_INST_VALU / CUs / GRBM_GUI_ACTIVE); wave_cycles: '
                                'SQ_* cycles / SQ_WAVE_CYCLES (WAIT_ANY = parked on s_waitcnt / barriers, '
                                'WAIT_INST_ANY = waiting to issue)'}
    if hot:
        roof['ops_per_candidate_draw'] = DRAW_OPS_PER_CAND
        roof['candidates_per_s'] = scr[0] / (dom_ms * 1e-3)
        roof['note'] = ('VALU-issue bound on integer work: achieved counts the draw\'s algorithmic 32-bit '
                        'lane operations (Philox4x32-10: 40 per candidate; the pick 4; the u-cell bit 3) '
                        'over the kernel\'s HIP-event time, against the 32-bit VALU lane rate; the fp64 '
                        'draws of the marked candidates (k_hot_draw) and the expansion screen of the listed '
                        'ones (k_screen_hot) are other_dense_ms; the PMC figures are k_hot_bx\'s')
    elif smode == 3:
        roof['flops_per_candidate_poly'] = BX_FLOPS_PER_CAND
        roof['note'] = ('VALU-issue bound: per candidate the Philox + Box-Muller draw, the fp64 '
                        'exp / log sequences and the bound take most of the instruction stream; '
                        'achieved counts only the lpdf arithmetic (6 FLOP per direct term, 40 per '
                        'polynomial); valu_busy_measured is the PMC utilisation of the same kernel')
    line = {
        'metric': 'TPE candidate x component lpdf evals/sec (10k-trial history)',
        # n_gpus: the distinct GPUs the ranks ran on (ranks sharing one card
        # -- the gloo rehearsals -- count it once; rccl_world counts ranks)
        'value': value, 'unit': 'evals/s', 'n_gpus': len(set(devs)) if devs else distinct_gpus(rank_devices),
        'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'strong', 'vs_baseline': None,
        'dtype': ('f32+f64' if screened else args.precision),
        'data': 'synthetic (prior draws, seed 0)',
        'rccl_world': world, 'dist_backend': args.dist_backend if dist is not None else None,
        'rank_devices': rank_devices, 'distinct_gpus': len(set(devs)) if devs else distinct_gpus(rank_devices),
        'value_only': bool(value_only),
        'config': {'workload': workload_name(args, C),
                   'labels': L, 'history': args.trials,
                   'candidates_per_label': C_total, 'candidates_per_label_per_gpu': C,
                   'parallelism': ('descriptor exchange x%d (posteriors of label shards %s all-gathered; '
                                   '%s)' % (world, [len(sh) for sh in shards],
                                            'new_id shards' if args.config == 5 else 'candidate shards')
                                   if desc else
                                   'label-sharded x%d (labels per rank: %s)'
                                   % (world, [len(sh) for sh in shards]) if by_label and world > 1 else
                                   ('new_id-sharded x%d' if args.config == 5
                                    else 'candidate-sharded x%d') % (len(devs) if devs else world))
                                  + (' (one process, multi-device context %s)' % devs
                                     if devs else '')},
        'step': ({'kind': 'fresh posterior (fmin loop)',
                  'note': 'each step appends %d trial(s) to the device-resident history, rebuilds the '
                          'posterior on the device (split, Parzen, fold; numpy\'s np.argsort tie order '
                          'where a mixture depends on it), builds the expansion index of the new '
                          'posterior and runs the round -- what every suggestion of fmin(tpe.suggest) '
                          'pays (reference: tpe_transform + rec_eval per call, tpe.py:834,900)'
                          % args.append,
                  'history_first_step': args.trials + args.append,
                  'expansion_index_ms': round(scr[7] / args.steps, 3),
                  'advance_breakdown_ms': {k: round(v[1] / args.steps * 1e3, 3)
                                           for k, v in sorted(phases.items())},
                  'advance_breakdown_note': 'host wall ms per step: append (transform + upload of the '
                                            'new observations), build (device build + its tie report, '
                                            'synchronous), prepare_enqueue (the expansion index queued), '
                                            'argsorts (numpy np.argsort for tie-dependent labels, while '
                                            'the index runs), rebuild (those labels again), round; with '
                                            'the dense labels\' round under the argsorts: '
                                            'argsorts_under_round (max of the two), rebuild, quant_round '
                                            '(the quantized labels after their rebuild); step_total = '
                                            'all of it',
                  'warm_round_ms': round(wdt / args.steps * 1e3, 3),
                  'warm_note': 'the same rounds on one resident posterior (no append, no rebuild, '
                               'no index): the round alone'}
                 if fresh_mode else
                 {'kind': 'warm (one resident posterior)',
                  'fresh_posterior_round_ms': (round(post_build['device_call_ms'] + prep_ms
                                                     + dt / args.steps * 1e3, 3) if prep_ms else None)}),
        'scaling_projection': proj,
        'scaling_projection_descriptors': dproj,
        'device_memory': mem,
        'posterior_build': dict(post_build, expansion_index_ms=(round(prep_ms, 3) if prep_ms else None),
                                expansion_index_note='the first index of the run (bin tables, lists, '
                                'sub-bin bounds; wall ms with the kernels)'),
        'per_family_ms': {k: round(v / args.steps, 3) for k, v in mode_ms.items() if v},
        'per_family_evals': {k: v // args.steps for k, v in mode_ev.items() if v},
        'roofline': roof,
        'evals_basis': {
            'value': 'executed terms per second, whole job',
            'executed_per_step': executed_all // max(args.steps, 1),
            'reference_equivalent_per_step': ref_equiv_per_step,
            'reference_equivalent_per_s': ref_equiv_per_step * args.steps / dt,
            'note': 'reference_equivalent: every (candidate, component) pair of the step '
                    '(C x (K_b + K_a) per numeric label, 2 C per categorical) -- the terms the '
                    'reference\'s GMM1_lpdf / LGMM1_lpdf / categorical_lpdf evaluate for the '
                    'same candidates, i.e. the step\'s work at the cpu_baseline\'s counting'},
    }
    if screened:
        line['screen'] = {
            'screened_per_step': scr[0] // args.steps, 'rescored_per_step': scr[1] // args.steps,
            'rescore_terms_per_step': scr[4] // args.steps,
            'rescored_fraction': scr[1] / max(scr[0], 1),
            'screen_kernel_ms': round(scr[2] / args.steps, 3),
            'other_dense_ms': round((mode_ms[dom] - scr[2]) / args.steps, 3),
            'windowed': windowed,
            'mode': {0: 'none', 1: 'plain fp32', 2: 'windowed fp32', 3: 'expansion (fp64)'}[smode],
            'screen_terms_per_step': scr[3] // args.steps,
            'hot_listed_per_step': scr[5] // args.steps,
            'hot_listed_fraction': scr[5] / max(scr[0], 1),
            'hot_fallbacks': scr[6],
            'screen_terms_fraction': scr[3] / max(mode_ev[dom], 1),
            'note': 'dense labels: every (candidate, component) pair is either evaluated in '
                    'packed fp32 with a rigorous error bound, or (windowed screen: candidates '
                    'sorted into tiles of neighbours) proven below 2^-T (win_t) of the largest term and '
                    'covered by the bound; candidates whose bound interval reaches the '
                    'round\'s best lower bound are re-scored in fp64 over every component -- '
                    '(expansion screen: fp64 score, bound ~1e-12, so only near-ties) -- '
                    'winners and lpdfs are bit-identical to the plain fp64 round '
                    '(tests/test_screen.py).  `value` counts the terms executed (screen + '
                    're-score); the roofline counts the terms the screening kernel summed.  '
                    'other_dense_ms: keys + sort, select, re-score'}
        if unscreened is not None:
            same, udt, nu, first, u_ms, u_ev = unscreened
            if u_ms > 0:
                line['roofline_lpdf'] = roofline_lpdf(u_ms / nu, u_ev / nu, args)
            line['screened_equals_fp64'] = bool(same)
            line['screen']['unscreened_fp64'] = {
                'steps': nu, 'ms_per_step': round(udt / nu * 1e3, 3),
                'compared': ('index and value (value-only rounds: a certified cell carries no '
                             'lpdfs)' if value_only else
                             'index, value, score, lpdf_below, lpdf_above, status') +
                            ' of every label, bytewise, on rounds %d..%d of the last posterior (the '
                            'screened runs are the warm steps)' % (first, first + nu - 1),
                'bit_identical': bool(same)}
    if prec == 'f32' and args.agreement_steps > 0 and args.config != 5:
        # fp32 winners vs the exact fp64 round's on the same candidate sets
        ref = Engine(devs if devs else local, 'f64')
        if loop is not None:   # the posterior the fp32 engine holds now
            FminLoop(hist_full, label_ids=loop.label_ids if loop.streams else None).advance(ref, loop.n)
        else:
            ref.build_posterior(*inputs, gamma=0.25, prior_weight=1.0)
        same = total = 0
        worst_regret = 0.0
        for i in range(args.agreement_steps):
            a = eng.suggest(seed=1234 + i, n_candidates=C, round=i, cand_offset=rank * C)
            b = ref.suggest(seed=1234 + i, n_candidates=C, round=i, cand_offset=rank * C)
            same += int(np.sum(a['index'] == b['index']))
            total += len(a)
            # regret in exact score of the fp32 winner (re-scored in fp64)
            for li in np.nonzero(a['index'] != b['index'])[0]:
                if posts[li].family == 'categorical':
                    continue
                lb, la, _ = ref.score(int(li), np.array([a[li]['value']]))
                worst_regret = max(worst_regret, float(b[li]['score'] - (lb[0] - la[0])))
        ref.close()
        line['f32_argmax_agreement'] = {
            'rate': same / max(total, 1), 'winners_compared': total,
            'worst_fp64_score_regret': worst_regret,
            'note': 'per (step, label): the fp32 round\'s winner index equals the exact fp64 '
                    'round\'s on the same candidates; regret = fp64 score of the fp64 winner '
                    'minus fp64 score of the fp32 winner'}
    if args.config == 5:
        line['config']['new_ids_per_step'] = args.new_ids
        line['config']['new_ids_per_gpu_per_step'] = ids_local
    if rank == 0 and not args.no_latency and args.config == 3:
        lat = suggest_latency(args.labels, args.trials)
        line['suggest_latency_ms'] = {
            'value': round(lat, 3), 'n_EI_candidates': 24, 'history': args.trials,
            'labels': args.labels, 'note': 'end-to-end tpe.suggest wall time, median of 20; '
                                           'reference CPU: 1330 ms (BASELINE.md)'}
    if rank == 0 and not args.no_latency and args.config == 3:
        wall, bx = config1_fmin()
        line['config1_fmin'] = {
            'wall_s': round(wall, 4), 'trials': 100, 'n_EI_candidates': 24, 'best_x': bx,
            'reference_cpu_s': 0.141,
            'note': 'BASELINE config 1: fmin(tpe.suggest) on the 1-D hp.uniform quadratic, 100 trials '
                    '(20 random startup + 80 TPE suggestions), RandomState(0), objective included; '
                    'median of 3 runs; every TPE suggestion is the oracle argmax of its 24 '
                    'candidates (tests/test_config1.py)'}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == 3:
        rate, sec, ev, thr = cpu_baseline_c(eng, posts, args.cpu_sample_c, 1234, 0)
        nrate, nsec, nev = cpu_baseline_numpy(posts, args.cpu_sample)
        line['cpu_baseline'] = {
            'value': rate, 'unit': 'evals/s', 'cores': thr, 'kind': 'port',
            'sample': 'the first %d of the 2^%d candidates of all %d labels (the GPU round\'s '
                      'own draws), scored under l and g and argmaxed by oracle/tpe_score.c, '
                      'the C restatement of tpe.py, OpenMP on %d threads; %.1f s, %.3g evals'
                      % (args.cpu_sample_c, args.cand_log2, L, thr, sec, ev),
            'single_core_numpy': {
                'value': nrate, 'cores': 1,
                'sample': 'all %d labels x %d candidates sampled, scored and argmaxed by the '
                          'numpy restatement (oracle/tpe_oracle.py); %.1f s, %.3g evals'
                          % (L, args.cpu_sample, nsec, nev)}}
    if agree_leg is not None:
        line['oracle_batched_agree' if args.config == 5 else 'oracle_near_tie_agree'] = agree_leg
    if others is not None:
        line['other_configs'] = others
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
