# round 2, call J: LDS-staged flatten + JIT sizing in the flatten pass + word-based JIT layout/emit:
# build-chain equality tests, GPU suite, bench, kernel trace
set -o pipefail
O=gpurun_out/r02j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_build.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py --no-pmc > $O/bench.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt -o kt -- python3 scripts/kprof.py --iters 5 > $O/kt.log 2>&1
echo "exit $?"
