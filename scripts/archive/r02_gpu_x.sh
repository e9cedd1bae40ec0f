# round 2, call X: table-driven wave JIT sizing, node counts stored by the flattener, templates in the emit kernel, sampled plan readback
set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_api.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_build.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 5 > $O/kt.log 2>&1
echo "exit $?"
