set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_c3_bench.log 2>&1
echo rc=$?
