# sourced by the scripts/gpu_r5_*.sh runners: `soft CMD...` lets a step fail with test failures
# (exit 1) and go on, but ends the script on anything else (a fault, an abort, a time limit)
soft() {
  local rc=0
  "$@" || rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "step failed with rc=$rc: $*" >&2
    exit $rc
  fi
  return 0
}
