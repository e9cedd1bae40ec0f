set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u scripts/kvariants.py --variants prod,nointerp --rounds 5 > gpurun_out/kv_nointerp.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/pmc1 -o pmc1 -- python3 scripts/kprof.py --iters 1 > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES -d gpurun_out/pmc2 -o pmc2 -- python3 scripts/kprof.py --iters 1 > gpurun_out/pmc2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/pmc3 -o pmc3 -- python3 scripts/kprof.py --iters 1 --lib multitreegp_amd/lib/variants/libmtgp_hip_nointerp.so > gpurun_out/pmc3.log 2>&1
