set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_value_only.py > gpurun_out/r4al_pytest.log 2>&1
