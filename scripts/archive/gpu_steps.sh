#!/bin/bash
# Run a list of named GPU steps from a file: "<name> <timeout> <command...>" per line.
# Stops at the first crash/timeout (exit > 1); test failures (exit 1) continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
while read -r name to cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  echo "== $name: $cmd"
  eval timeout -k 10 "$to" $cmd > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"; grep -v "amdgpu.ids\|simple_timer\|output_stream\|tool.cpp" "gpurun_out/$name.log" | tail -n 12
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < "$1"
