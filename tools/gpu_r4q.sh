# round-4: the whole GPU suite, smoke, then the default bench line
set -o pipefail
O=gpurun_out/${R4OUT:-r4q}
mkdir -p $O/nt
NEAR_TIE_OUT=$O/nt timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py > $O/bench.log 2>&1
