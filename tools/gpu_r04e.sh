# Round 4 (re-entry): idle-gap relaunch split at the lanes code, the control plane
# (RCCL tick tests, idle ticks, alloc latency with the hop split), the shared-GPU
# rehearsal test, then the N=1 bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r04e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/idle_gap_probe.py --variants default,idle200 --out $OUT/idle_gap.json > $OUT/idle_gap.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ctrl.log 2>&1 &&
timeout -k 10 300 python3 -u tools/idle_tick_probe.py --repeat 2 --out $OUT/idle_tick.json > $OUT/idle_tick.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ctrl_probe.py --variants tcp,rccl_tick,rccl_idle0 --repeat 3 --out $OUT/ctrl_probe.json > $OUT/ctrl_probe.log 2>&1 &&
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_share.py -m gpu -v -s --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_share.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json > $OUT/bench_n1.log 2>&1
rc=$?; cat $OUT/idle_gap.log | cut -c1-400; tail -3 $OUT/pytest_ctrl.log; tail -c 1500 $OUT/idle_tick.log; tail -c 600 $OUT/ctrl_probe.log; tail -3 $OUT/pytest_share.log; tail -c 300 $OUT/bench_n1.log; exit $rc
