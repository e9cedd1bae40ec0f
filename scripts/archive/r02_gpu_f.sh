# round 2, call F: fallback diagnosis -- trig v2 with (inline) and without (nofb) the interpreter re-run
set -o pipefail
O=gpurun_out/r02f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kvariants.py --variants base,inline,nofb --rounds 6 > $O/ab_fb.log 2>&1
echo "exit $?"
