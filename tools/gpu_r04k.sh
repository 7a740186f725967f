# Round 4: RCCL tick tests and the control-plane probe after dropping the per-tick
# event; the 8-rank one-GPU rehearsal with HIP lanes and with no lone lead; the N=1
# bench under rocprofv3.
set -o pipefail
mkdir -p gpurun_out/r04k gpurun_out/s8hip gpurun_out/s8lone0 gpurun_out/prof_r04
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k/pytest_service.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k/pytest_ctrl.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ctrl_probe.py --variants tcp,rccl_tick --repeat 3 --out gpurun_out/r04k/ctrl_probe.json > gpurun_out/r04k/ctrl_probe.log 2>&1 &&
OUT=gpurun_out/s8hip PORT=29561 OCM_SERVICE_QUEUE=hip timeout -k 10 400 bash tools/gpu_share8.sh &&
OUT=gpurun_out/s8lone0 PORT=29571 OCM_SERVICE_LONE_US=0 timeout -k 10 400 bash tools/gpu_share8.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04 -o bench -- python3 -u bench.py --steps 5 --warmup 2 --json-out gpurun_out/prof_r04/bench.json > gpurun_out/prof_r04/bench.log 2>&1
rc=$?; tail -2 gpurun_out/r04k/pytest_service.log; tail -2 gpurun_out/r04k/pytest_ctrl.log; grep -E "alloc_p50" gpurun_out/r04k/ctrl_probe.log | head; find gpurun_out/prof_r04 -name "*kernel_stats.csv" | head -3; exit $rc
