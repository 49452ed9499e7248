#!/bin/bash
# round 6: the whole -m gpu suite, then the default bench line (calibration, extras, CPU baseline)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r6b}
( while true; do date >> gpurun_out/${TAG}_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -v -rf --timeout 1200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
echo "tests rc=$rc"
