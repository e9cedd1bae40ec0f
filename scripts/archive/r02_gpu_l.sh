# round 2, call L: flatten lanes-per-block A/B (MTGP_FLAT_LANES 32 / 16 / 8), kernel trace each
set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_build.log 2>&1 && \
for L in 32 16 8; do
  MTGP_FLAT_LANES=$L timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt$L -o kt -- python3 scripts/kprof.py --iters 5 > $O/kt$L.log 2>&1 || exit 1
done
echo "exit $?"
