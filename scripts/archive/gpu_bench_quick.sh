set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bq_jit.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --obs-noise 0.1 > gpurun_out/bq_jit_noise.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traj > gpurun_out/bq_jit_fit.log 2>&1
