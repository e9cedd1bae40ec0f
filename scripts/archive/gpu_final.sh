set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/final_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --obs-noise 0.1 > gpurun_out/final_c3_noise.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --rollouts 16 --pop 1024 > gpurun_out/final_c2.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config c5 --rollouts 8 --pop 4096 --steps 3 --warmup 1 > gpurun_out/final_c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o c3 --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_final_bench.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f --output-format csv -- python3 scripts/kprof.py --iters 2 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w --output-format csv -- python3 scripts/kprof.py --iters 2 > gpurun_out/pmc_write.log 2>&1
echo rc=$?
