# round 2, call B: notebook pins + full-size parity on the GPU
set -o pipefail
O=gpurun_out/r02b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_notebook_pin.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_pin_full.log 2>&1
echo "exit $?"
