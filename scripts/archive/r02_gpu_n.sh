# round 2, call N: role-chained JIT (ABI v13): GPU suite, smoke, A/B (chained / one call per program /
# environment only), C3 bench with live PMC, rocprof kernel stats, SQ issue counters
set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_build.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants prod,prod@MTGP_JIT_CHAIN=0,noprog@MTGP_JIT_CHAIN=0 --rounds 6 > $O/ab_chain.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 3 > $O/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/ps1 -o ps1 -- python3 scripts/kprof.py --iters 1 > $O/ps1.log 2>&1
echo "exit $?"
