# round 2, call M: LDS-mode JIT for the wide-state SR kernel (C5): build-chain tests, GPU suite, C5 + C3 bench
set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_build.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc > $O/bench_c5.log 2>&1 && \
MTGP_JIT=0 timeout -k 10 600 python bench.py --config c5 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline > $O/bench_c5_interp.log 2>&1 && \
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $O/bench_c3.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt5 -o kt -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 3 > $O/kt5.log 2>&1
echo "exit $?"
