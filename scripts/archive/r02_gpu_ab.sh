# round 2, call AB: single-wave flatten blocks restored, node counts by atomics for many trees (C5):
# GPU suite, smoke, C3 / C5 bench, C3 and C5 kernel stats
set -o pipefail
O=gpurun_out/r02ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc --no-cpu-baseline > $O/bench_c5.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 5 > $O/kt.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 -- python3 scripts/kprof.py --iters 3 --config c5 > $O/kt5.log 2>&1
echo "exit $?"
