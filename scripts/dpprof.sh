set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dpprof; mkdir -p $O
for b in 0 100 500; do
  MTGP_DP_BUDGET=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/b$b -o b$b -- python3 scripts/kprof.py --iters 4 --config c3 --solver dopri5 > $O/b$b.log 2>&1 || exit 1
  f=$(find $O/b$b -name '*kernel_stats.csv' | head -1); echo "== budget $b"; head -4 $f | cut -c1-200
  f2=$(find $O/b$b -name '*kernel_trace.csv' | head -1); grep k_ctl_dopri5 $f2 | awk -F, '{print $0}' | head -12 | cut -c1-50 > /dev/null
done
