# round 2, call G: trig v2 templates with out-of-line slow blocks: jit_smoke sweep, GPU suite, A/B, bench
set -o pipefail
O=gpurun_out/r02g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/jit_smoke > $O/jit_smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants base,prod --rounds 6 > $O/ab_trig.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
echo "exit $?"
