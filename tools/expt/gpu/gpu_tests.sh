#!/bin/bash
# GPU-box helper: pytest -m gpu on the given test files (default: all), log
# under gpurun_out/${OUT:-tests}/pytest.log.
set -o pipefail
O=gpurun_out/${OUT:-tests}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -15
tail -3 $O/pytest.log
exit $rc
