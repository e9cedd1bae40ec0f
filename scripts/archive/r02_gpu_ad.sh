# round 2, call AD: final tree of the round -- GPU suite, smoke, C3 driver bench
set -o pipefail
O=gpurun_out/r02ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1
echo "exit $?"
