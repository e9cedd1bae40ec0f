# round 2, call I: coefficient optimisation (mtgp_sr_grad) + the whole GPU suite
set -o pipefail
O=gpurun_out/r02i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "exit $?"
