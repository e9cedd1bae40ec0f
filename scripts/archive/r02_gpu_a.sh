# round 2, call A: GPU suite + bench + HEAD PMC (traffic + issue counters) for the C3 kernel
set -o pipefail
O=gpurun_out/r02a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 3 > $O/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pf -- python3 scripts/kprof.py --iters 1 > $O/pf.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pw -- python3 scripts/kprof.py --iters 1 > $O/pw.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/ps1 -o ps1 -- python3 scripts/kprof.py --iters 1 > $O/ps1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/ps2 -o ps2 -- python3 scripts/kprof.py --iters 1 > $O/ps2.log 2>&1
echo "exit $?"
