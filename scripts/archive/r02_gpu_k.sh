# round 2, call K: PMC passes over the per-population build chain (flatten, JIT sizes/scan/emit)
set -o pipefail
O=gpurun_out/r02k; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/ps1 -o ps1 -- python3 scripts/kprof.py --iters 2 > $O/ps1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/ps2 -o ps2 -- python3 scripts/kprof.py --iters 2 > $O/ps2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT -d $O/ps3 -o ps3 -- python3 scripts/kprof.py --iters 2 > $O/ps3.log 2>&1
echo "exit $?"
