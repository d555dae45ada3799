# round-4: R = 6 product -- the screen / fmin-loop / full-size tests, then the profile set
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_screen.py tests/test_fmin_loop.py tests/test_gpu_fullsize.py tests/test_near_tie_agreement.py > gpurun_out/r4ak_pytest.log 2>&1 || exit 1
bash tools/prof_round.sh r4ak --steps 5 --warmup 2 --no-other-configs --no-agreement
