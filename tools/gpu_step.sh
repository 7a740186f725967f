set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ctrl_tick.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 && \
timeout -k 10 400 python -u tools/ctrl_probe.py --variants rccl_tick_ring_hbm --repeat 1 --out gpurun_out/ctrl_probe_ring.json > gpurun_out/ctrl_probe_ring.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_step.log; python3 -c "
import json; d=json.load(open('gpurun_out/ctrl_probe_ring.json'))
for k,v in d.items(): print(k, v['alloc_p50_us'], v['alloc_p99_us'], v['free_p50_us'], v['ticks'], v.get('daemon_log'))
"; grep -i warn gpurun_out/ctrl_probe_ring.log | head -3; exit $rc
