# round 2, call S: two programs per wave in the flattener (N <= 64), fused single-block schedule,
# register-resident JIT size scan: build-chain equality + full-size parity + GPU suite, flatten A/B
# (2 / 1 programs per wave / lane-per-program) with the flatten timed, C3 bench, rocprof stats
set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_fullsize.py tests/test_gpu_schedule.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_build_full.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants prod,prod@MTGP_FLAT_PPW=1,prod@MTGP_FLAT_MODE=lane --rounds 10 --reflatten > $O/ab_flat_c3.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 10 > $O/kt.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 3 > $O/kt5.log 2>&1
echo "exit $?"
