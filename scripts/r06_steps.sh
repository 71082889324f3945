#!/bin/bash
# round 6: GPU call runner.  Each step is "name|seconds|command"; output in gpurun_out/r06$TAG/<name>.log.
# A step that fails normally (a test failure, exit 1/2/3) lets the next one run; a time limit, an abort
# or a signal (124, 134, 137, 139, >128) ends the call there -- nothing more starts on the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r06${TAG}
mkdir -p $OUT
worst=0
while IFS= read -r spec; do
  [ -z "$spec" ] && continue
  case "$spec" in \#*) continue ;; esac
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($secs s): $cmd" | tee -a $OUT/steps.txt
  t0=$(date +%s)
  timeout -k 10 $secs bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "=== $name: exit $rc after $(( $(date +%s) - t0 )) s" | tee -a $OUT/steps.txt
  tail -3 $OUT/$name.log
  [ $rc -ne 0 ] && worst=$rc
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== stopping: step $name ended with $rc" | tee -a $OUT/steps.txt
    exit $rc
  fi
done < "${1:-/dev/stdin}"
exit $worst
