# Service stream priority: sweep trace (torch + verify), loopback bench, service tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/sweep_trace.py --remote loopback --torch --verify > gpurun_out/st_both_prio.json 2> gpurun_out/st_both_prio.err && \
timeout -k 10 200 python -u bench.py --remote loopback --no-optim-extra --json-out gpurun_out/bench_loop_prio.json > gpurun_out/bench_loop_prio.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_prio.log 2>&1
rc=$?
python3 -c "
import json
d=json.load(open('gpurun_out/st_both_prio.json')); print('trace', [s['step_ms'] for s in d['steps']])
b=json.load(open('gpurun_out/bench_loop_prio.json')); print('loop', b['value'], b['ms_per_step'])
"; tail -1 gpurun_out/pytest_prio.log; exit $rc
