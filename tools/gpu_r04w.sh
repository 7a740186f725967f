# Round 4: RCCL idle ticks wait on the GPU only within 2 ms of traffic. The RCCL tick
# GPU tests, then the idle-tick probe with a GEMM on the same GPU while the mesh idles.
set -o pipefail
OUT=${OUT:-gpurun_out/r04w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ctrl.log 2>&1 &&
timeout -k 10 600 python3 -u tools/idle_tick_probe.py --repeat 2 --out $OUT/idle_tick.json > $OUT/idle_tick.log 2>&1
rc=$?; tail -2 $OUT/pytest_ctrl.log; grep -E "FAILED|ERROR" $OUT/pytest_ctrl.log | head; cut -c1-260 $OUT/idle_tick.log; exit $rc
