# round 2, call H (re-entry): HEAD rebuilt from source -- GPU suite, smoke, bench (live PMC), kernel trace stats
set -o pipefail
O=gpurun_out/r02h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 3 > $O/kt.log 2>&1
echo "exit $?"
