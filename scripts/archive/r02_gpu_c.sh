# round 2, call C: env-only vs base A/B; icache / branch counters of the C3 kernel
set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kvariants.py --variants base,noprog --rounds 5 > $O/ab_noprog.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_BRANCH SQ_WAVES -d $O/pi -o pi -- python3 scripts/kprof.py --iters 1 > $O/pi.log 2>&1
echo "exit $?"
