# Round 4: the RCCL tick GPU tests with the idle-seal window test.
set -o pipefail
OUT=${OUT:-gpurun_out/r04y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ctrl.log 2>&1
rc=$?; tail -2 $OUT/pytest_ctrl.log; grep -E "FAILED|ERROR|idle ticks waited|window" $OUT/pytest_ctrl.log | head; exit $rc
