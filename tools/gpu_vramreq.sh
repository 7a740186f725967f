# VRAMREQ (protocol bit 64): the copy service's request records in fine-grained
# HBM written by the CPU through the BAR, against host memory (default 15):
# service GPU tests under 79, then interleaved bench.py sweeps (host tier to
# 16 MiB, loopback HBM to 4 MiB).
set -o pipefail
OUT=${OUT:-gpurun_out/vramreq}
mkdir -p $OUT
timeout -k 10 400 env OCM_SERVICE_PROTO=79 python3 -u -m pytest tests/test_gpu_service.py tests/test_gpu_runtime.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2 3; do
  for p in 15 79; do
    timeout -k 10 200 env OCM_SERVICE_PROTO=$p python3 -u bench.py --steps 10 --warmup 3 --max-bytes 16777216 --no-optim-extra --no-ctrl-extra --json-out $OUT/host_p${p}_$i.json > $OUT/host_p${p}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for p in 15 79; do
    timeout -k 10 200 env OCM_SERVICE_PROTO=$p python3 -u bench.py --remote loopback --steps 10 --warmup 3 --max-bytes 4194304 --no-optim-extra --no-ctrl-extra --json-out $OUT/hbm_p${p}_$i.json > $OUT/hbm_p${p}_$i.log 2>&1 || exit $?
  done
done
grep -l "stay in host memory" $OUT/*.log || echo "no fallback warnings"
python3 - <<'PY'
import json, glob, os
out = os.environ.get('OUT', 'gpurun_out/vramreq')
for f in sorted(glob.glob(out + '/*.json')):
    d = json.load(open(f)); sw = d['sweep']
    print(os.path.basename(f), ' '.join(f"{int(s)>>10}K:{sw[s]['get_us']}/{sw[s]['put_us']}" for s in sw))
PY
