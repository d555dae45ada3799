# round-4: quantized-runs oracle test, then the final line + profile set
set -o pipefail
mkdir -p gpurun_out/r4ar
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "quantized or fused or sampler" > gpurun_out/r4ar/pytest_q.log 2>&1 || exit 1
bash tools/gpu_r4ar.sh
