# Round 4: the idle-gap relaunch split, the control plane (RCCL tick tests, idle
# ticks vs TCP wake-ups, alloc latency with the hop breakdown, the GPU time idle
# ticks take), then the shared-GPU rehearsal test.
set -o pipefail
OUT=${OUT:-gpurun_out/r04d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/idle_gap_probe.py --out $OUT/idle_gap.json > $OUT/idle_gap.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ctrl.log 2>&1 &&
timeout -k 10 300 python3 -u tools/idle_tick_probe.py --repeat 2 --out $OUT/idle_tick.json > $OUT/idle_tick.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ctrl_probe.py --variants tcp,rccl_tick,rccl_idle0 --repeat 3 --out $OUT/ctrl_probe.json > $OUT/ctrl_probe.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o idle -- python3 -u tools/idle_tick_probe.py --modes 1000 --repeat 1 > $OUT/idle_prof.log 2>&1 &&
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_share.py -m gpu -v -s --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_share.log 2>&1
rc=$?; cat $OUT/idle_gap.log | cut -c1-400; tail -3 $OUT/pytest_ctrl.log; tail -c 1500 $OUT/idle_tick.log; tail -c 600 $OUT/ctrl_probe.log; tail -3 $OUT/pytest_share.log; exit $rc
