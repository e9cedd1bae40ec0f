# round 2, call Q: C5 A/B (wave / lane flatten, store chains on / off) with the flatten timed, C3 + C5
# bench, rocprof kernel stats of both (call P ran the suites: build/full-size 21/21, GPU 138/138)
set -o pipefail
O=gpurun_out/r02q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kvariants.py --config c5 --variants prod,prod@MTGP_FLAT_MODE=lane,prod@MTGP_JIT_CHAIN=0 --rounds 4 --reflatten > $O/ab_c5.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc > $O/bench_c5.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 10 > $O/kt.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 3 > $O/kt5.log 2>&1
echo "exit $?"
