# round 2, call E: GPU suite; A/B old trig (base) / trig v2 (prod) / trig v2 inlined (inline); bench with live PMC
set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants base,prod,inline --rounds 6 > $O/ab_trig.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
echo "exit $?"
