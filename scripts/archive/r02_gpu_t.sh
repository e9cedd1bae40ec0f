# round 2, call T: pipelined LDS-data JIT units (preloads of the next group issued before the current
# group's body), one program per wave in the flattener again, fused schedule for small P * n_prog,
# register-resident size scan: build-chain equality + full-size parity + GPU suite, C5 A/B
# (pipelined / not), C3 + C5 bench, rocprof stats, SQ counters of the C5 kernel
set -o pipefail
O=gpurun_out/r02t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_fullsize.py tests/test_gpu_schedule.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_build_full.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --config c5 --variants prod,prod@MTGP_JIT_LDS_PIPE=0 --rounds 4 > $O/ab_pipe_c5.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc > $O/bench_c5.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 10 > $O/kt.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 3 > $O/kt5.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/ps5 -o ps5 -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 1 > $O/ps5.log 2>&1
echo "exit $?"
