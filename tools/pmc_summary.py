"""Summarise one tools/prof_round.sh output directory into profiles/:

    python tools/pmc_summary.py gpurun_out/r1c r1c

writes profiles/<tag>_kernel_stats.csv, <tag>_domain_stats.csv (copies of the
rocprofv3 --stats tables), <tag>_bench.json (the bench line), and
<tag>_pmc_summary.json: per kernel, each PMC counter averaged PER LAUNCH
(FETCH_SIZE / WRITE_SIZE in KB as rocprofv3 reports them), plus for the dense
round kernels the VALU instructions per eval (evals per launch from the bench
line's per_family_evals over the bench's launches of that kernel; for the
windowed k_screen_win the terms it summed, screen.screen_terms_per_step)."""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

FAMILY = {'k_screen<': 'dense',
          'k_round<double, 0,': 'dense', 'k_round<double, 1,': 'dense_lgmm1',
          'k_round<float, 0,': 'dense', 'k_round<float, 1,': 'dense_lgmm1',
          'k_round<double, 8,': 'dense', 'k_round<float, 8,': 'dense'}


def short(name):
    name = re.sub(r'^(void )?\(anonymous namespace\)::', '', name)
    name = re.sub(r'^void ', '', name)
    depth, out = 0, []
    for ch in name:     # cut the argument list, keep template arguments
        if ch == '<':
            depth += 1
        elif ch == '>':
            depth -= 1
        elif ch == '(' and depth == 0:
            break
        out.append(ch)
    return ''.join(out).strip()


def pmc(path):
    per = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    dur = defaultdict(dict)
    for row in csv.DictReader(open(path)):
        k = short(row['Kernel_Name'])
        per[k][row['Counter_Name']] += float(row['Counter_Value'])
        launches[k].add(row['Dispatch_Id'])
        if row.get('Start_Timestamp') and row.get('End_Timestamp'):
            dur[k][row['Dispatch_Id']] = float(row['End_Timestamp']) - float(row['Start_Timestamp'])
    out = {k: {c: v / len(launches[k]) for c, v in d.items()} for k, d in per.items()}
    for k, d in dur.items():   # the launch duration IN THIS (counter) run
        out[k]['_pmc_run_ns_per_launch'] = sum(d.values()) / len(d)
    return out, {k: len(v) for k, v in launches.items()}


def main(src, tag):
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles')
    for kind in ('kernel_stats', 'domain_stats'):
        f = glob.glob(os.path.join(src, 'trace', '*%s.csv' % kind))
        if f:
            shutil.copy(f[0], os.path.join(dst, '%s_%s.csv' % (tag, kind)))
    bench = None
    log = os.path.join(src, 'bench.log')
    if os.path.exists(log):
        for line in open(log):
            if line.startswith('{"metric"'):
                bench = json.loads(line)
        if bench:
            json.dump(bench, open(os.path.join(dst, '%s_bench.json' % tag), 'w'))
    summary, nlaunch = defaultdict(dict), {}
    for f in sorted(glob.glob(os.path.join(src, 'pmc_*', '*counter_collection.csv'))):
        d, n = pmc(f)
        for k, v in d.items():
            summary[k].update(v)
            nlaunch[k] = n[k]
    # evals per launch of each dense family from a 1-step bench line
    pmc_bench = os.path.join(src, 'pmc_valu.log')
    fam_evals, steps, win_terms, cands = None, 1, None, None
    if os.path.exists(pmc_bench):
        for line in open(pmc_bench):
            if line.startswith('{"metric"'):
                d = json.loads(line)
                fam_evals = d.get('per_family_evals')
                steps = d.get('steps', 1) + d.get('warmup', 0)   # every step launches once
                # the windowed screen's own terms (it skips the negligible pairs)
                win_terms = d.get('screen', {}).get('screen_terms_per_step')
                cands = d.get('screen', {}).get('screened_per_step')
    for k, v in summary.items():
        v['_launches'] = nlaunch.get(k)
        for pre, fam in FAMILY.items():
            if k.startswith(pre) and fam_evals and fam in fam_evals and 'SQ_INSTS_VALU' in v:
                # evals per launch = family evals per step x steps / launches
                ev = fam_evals[fam] * steps / max(nlaunch.get(k, 1), 1)
                v['_evals_per_launch'] = ev
                v['_valu_instr_per_eval'] = v['SQ_INSTS_VALU'] * 64 / ev
        if k.startswith('k_screen_win') and win_terms and 'SQ_INSTS_VALU' in v:
            ev = win_terms * steps / max(nlaunch.get(k, 1), 1)
            v['_evals_per_launch'] = ev
            v['_valu_instr_per_eval'] = v['SQ_INSTS_VALU'] * 64 / ev
        if k.startswith(('k_screen_bx', 'k_hot_bx')) and cands and 'SQ_INSTS_VALU' in v:
            # the expansion screen / hot prefilter: VALU instructions per
            # candidate (k_hot_bx: ONE launch per round over every dense
            # label's candidates, whatever extra rounds the run made)
            c = (cands if k.startswith('k_hot_bx')
                 else cands * steps / max(nlaunch.get(k, 1), 1))
            v['_candidates_per_launch'] = c
            v['_valu_instr_per_candidate'] = v['SQ_INSTS_VALU'] * 64 / c
        if 'SQ_INSTS_VALU' in v and v.get('GRBM_GUI_ACTIVE'):
            # VALU issue utilisation: every wave64 VALU instruction holds a
            # 16-lane SIMD for 4 cycles; 1024 SIMDs; GRBM_GUI_ACTIVE / 8 XCDs
            # = the launch's GPU cycles
            cycles = 1024 * v['GRBM_GUI_ACTIVE'] / 8
            v['_valu_busy'] = v['SQ_INSTS_VALU'] * 4 / cycles
            # the clock the counter run actually ran at: GPU cycles per XCD
            # over the launch's duration in that run (bench.py refuses PMC
            # figures from a run below 2 GHz)
            ns = v.get('_pmc_run_ns_per_launch')
            if ns:
                v['_eff_clock_ghz'] = v['GRBM_GUI_ACTIVE'] / 8 / ns
            if k.startswith('k_screen') and '_evals_per_launch' in v:
                # one v_exp_f32 (8-cycle issue) per eval: 4 extra cycles per
                # 64 evals on top of the 4-cycle count
                v['_valu_busy'] = (v['SQ_INSTS_VALU'] + v['_evals_per_launch'] / 64) * 4 / cycles
        if 'FETCH_SIZE' in v:
            v['_hbm_bytes_per_launch'] = (v['FETCH_SIZE'] * 2 + v.get('WRITE_SIZE', 0)) * 1024
    summary['_note'] = ('counters averaged per launch; FETCH_SIZE/WRITE_SIZE in KB; '
                        '_hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) KB per the gfx950 '
                        'FETCH_SIZE correction of MI355X_MICROARCH.md; SQ_INSTS_VALU counts wave '
                        'instructions (x64 lanes for _valu_instr_per_eval); GRBM_GUI_ACTIVE is '
                        'summed over the 8 XCDs; _valu_busy = SQ_INSTS_VALU x 4 cycles / '
                        '(1024 SIMDs x GRBM_GUI_ACTIVE / 8); _eff_clock_ghz = GRBM_GUI_ACTIVE / 8 / '
                        'the launch duration in the counter run (_pmc_run_ns_per_launch)')
    json.dump(summary, open(os.path.join(dst, '%s_pmc_summary.json' % tag), 'w'), indent=1,
              sort_keys=True)
    print(json.dumps({k: v for k, v in summary.items() if k.startswith(('k_round', 'k_screen'))},
                     indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
