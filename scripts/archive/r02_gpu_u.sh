# round 2, call U: RK4 bookkeeping branched on the uniform stage + finite-state observation fast path
# (A/B vs the same library without them, variants/base), GPU suite, smoke, C3 bench, rocprof stats
set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants prod,base --rounds 10 > $O/ab_stage.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-pmc --no-cpu-baseline > $O/bench_c2.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 10 > $O/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/ps1 -o ps1 -- python3 scripts/kprof.py --iters 1 > $O/ps1.log 2>&1
echo "exit $?"
