# round 2, call D: trig spec v2 (pi grid, branch-free JIT templates): GPU suite, A/B vs the
# pre-change library (variants/base), bench
set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants base,prod --rounds 6 > $O/ab_trig.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
echo "exit $?"
