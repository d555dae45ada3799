"""bench.py with module switches from the environment (A/B timing runs):
BENCH_SUBSET_REBUILD=0 turns the label-subset rebuild off (a variant of an
older commit has no tpe_rebuild_labels)."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hyperopt_amd.posterior as P  # noqa: E402

if os.environ.get('BENCH_SUBSET_REBUILD') == '0':
    P.SUBSET_REBUILD = False
sys.argv = ['bench.py'] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'bench.py'),
               run_name='__main__')
