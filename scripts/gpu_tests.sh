#!/bin/bash
# One gpurun call: the named GPU test files (default: all), each step time-limited, stop at the
# first failure that is a fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
rc=$?
tail -30 gpurun_out/tests.log
exit $rc
