# round 2, call AA: final state of the round -- GPU suite, smoke, every bench config, C3 and C3-Dopri5
# kernel stats, SQ issue counters of the C3 kernel
set -o pipefail
O=gpurun_out/r02aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-pmc --no-cpu-baseline > $O/bench_c2.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc --no-cpu-baseline > $O/bench_c5.log 2>&1 && \
timeout -k 10 300 python bench.py --obs-noise 0.1 --no-pmc --no-cpu-baseline > $O/bench_c3_noise.log 2>&1 && \
timeout -k 10 400 python bench.py --solver dopri5 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline > $O/bench_c3_dopri5.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 5 > $O/kt.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/ktd -o ktd -- python3 scripts/kprof.py --iters 2 --solver dopri5 > $O/ktd.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/ps1 -o ps1 -- python3 scripts/kprof.py --iters 1 > $O/ps1.log 2>&1
echo "exit $?"
