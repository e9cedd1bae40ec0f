set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/jit_smoke > gpurun_out/jit_smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --obs-noise 0.1 > gpurun_out/bench_c3_noise.log 2>&1 && \
timeout -k 10 200 python -u scripts/residency.py --jit 1 > gpurun_out/res.log 2>&1
