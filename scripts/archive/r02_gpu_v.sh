# round 2, call V: general PIDController (ABI v15): Dopri5 tests first, then GPU suite, smoke, bench
set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dopri5.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_dopri5.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
echo "exit $?"
