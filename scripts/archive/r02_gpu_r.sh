# round 2, call R: HEAD re-check after the wave flattener, LDS store chains and save counters:
# GPU suite, smoke, every bench config (C3 driver line with live PMC, C2, C5, C3 + obs noise,
# C3 Dopri5), rocprof kernel stats (C3 10 evaluations, C5, C3 Dopri5)
set -o pipefail
O=gpurun_out/r02r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-pmc > $O/bench_c2.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-pmc > $O/bench_c5.log 2>&1 && \
timeout -k 10 300 python bench.py --obs-noise 0.1 --no-pmc --no-cpu-baseline > $O/bench_c3_noise.log 2>&1 && \
timeout -k 10 400 python bench.py --solver dopri5 --steps 10 --warmup 2 --no-pmc > $O/bench_c3_dopri5.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/kprof.py --iters 10 > $O/kt.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 -- python3 scripts/kprof.py --config c5 --pop 4096 --rollouts 8 --iters 3 > $O/kt5.log 2>&1 && \
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/ktd -o ktd -- python3 scripts/kprof.py --solver dopri5 --iters 2 > $O/ktd.log 2>&1
echo "exit $?"
