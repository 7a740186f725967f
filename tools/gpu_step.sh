set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_runtime.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 && \
timeout -k 10 400 python -u tools/svc_probe.py --tiers host,hbm --configs default,hostget2 --out gpurun_out/svc_span2.json > gpurun_out/svc_span2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_step.log; python3 -c "
import json; d=json.load(open('gpurun_out/svc_span2.json'))
for k,v in d.items(): print(k, {s:(v[s]['get_us'],v[s]['put_us']) for s in ['4096','32768','65536','131072','262144','1048576','4194304'] if s in v})
" 2>/dev/null; exit $rc
