set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/residency.py --jit 1 > gpurun_out/res.log 2>&1 && \
timeout -k 10 200 python -u scripts/residency.py --jit 0 >> gpurun_out/res.log 2>&1
