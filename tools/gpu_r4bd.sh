# round-4: second pass of the whole GPU suite on the final tree
set -o pipefail
O=gpurun_out/r4bd
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
