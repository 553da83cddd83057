#!/bin/bash
# Every GPU test in one process per file group (the round-end driver runs `pytest -m gpu` the same way).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/alltests
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 240 --timeout-method thread tests/ > $O/test.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/test.log | tail -25
exit $rc
