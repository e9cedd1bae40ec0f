set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/pmcj1 -o pmcj1 -- python3 scripts/kprof.py --iters 1 > gpurun_out/pmcj1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_IFETCH SQ_BUSY_CYCLES -d gpurun_out/pmcj2 -o pmcj2 -- python3 scripts/kprof.py --iters 1 > gpurun_out/pmcj2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/pmcj3 -o pmcj3 -- python3 scripts/kprof.py --iters 1 > gpurun_out/pmcj3.log 2>&1
echo done
