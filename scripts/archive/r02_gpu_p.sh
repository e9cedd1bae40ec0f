# round 2, call P: wave-per-program flattener (k_flatten_wave) + LDS store chains for C5 (ABI v14): build-chain equality, full-size parity,
# GPU suite, flatten A/B (wave / lane) at C3 and C5 with the flatten inside the timed region,
# C3 bench (live PMC) + C5 bench, rocprof kernel stats of both
set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_build_full.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --variants prod,prod@MTGP_FLAT_MODE=lane,prod@MTGP_JIT_CHAIN=0 --rounds 8 --reflatten > $O/ab_flat_c3.log 2>&1 && \
timeout -k 10 300 python scripts/kvariants.py --config c5 --variants prod,prod@MTGP_FLAT_MODE=lane,prod@MTGP_JIT_CHAIN=0 --rounds 4 --reflatten > $O/ab_flat_c5.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc > $O/bench_c5.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 10 > $O/kt.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 3 > $O/kt5.log 2>&1
echo "exit $?"
