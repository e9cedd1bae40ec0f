#!/bin/bash
# One GPU session: parity tests -> smoke -> short bench -> rocprof kernel stats.
# Stops at the first crash/timeout (exit status > 1); a plain test failure (1) still
# lets the later steps run so the log shows everything.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py --steps 3 --warmup 1 --cpu-seconds 8
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
fi
