# Cost of the STRICT (peer-HBM) hand-off on the same-GPU stand-in: every request
# forced STRICT (OCM_SERVICE_STRICT=1) with the fenced plain copy (proto 15) or
# the write-through copy behind the acquire (STRICTWT, proto 47), against the
# default write-through hand-off, on a loopback HBM pair; the service GPU tests
# under both forced-STRICT forms first.
set -o pipefail
OUT=${OUT:-gpurun_out/strictwt}
mkdir -p $OUT
for p in 15 47; do
  timeout -k 10 400 env OCM_SERVICE_STRICT=1 OCM_SERVICE_PROTO=$p python3 -u -m pytest tests/test_gpu_service.py tests/test_gpu_runtime.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$p.log 2>&1 || { tail -30 $OUT/pytest_$p.log; exit 1; }
  tail -1 $OUT/pytest_$p.log
done
for i in 1 2 3; do
  for arm in default strict15 strict47; do
    case $arm in
      default) E="";;
      strict15) E="OCM_SERVICE_STRICT=1 OCM_SERVICE_PROTO=15";;
      strict47) E="OCM_SERVICE_STRICT=1 OCM_SERVICE_PROTO=47";;
    esac
    timeout -k 10 200 env $E python3 -u bench.py --remote loopback --steps 20 --warmup 3 --max-bytes 4194304 --no-optim-extra --no-ctrl-extra --json-out $OUT/${arm}_$i.json > $OUT/${arm}_$i.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get('OUT', 'gpurun_out/strictwt')
for f in sorted(glob.glob(out + '/*.json')):
    d = json.load(open(f)); sw = d['sweep']
    print(os.path.basename(f), ' '.join(f"{int(s)>>10}K:{sw[s]['get_us']}/{sw[s]['put_us']}" for s in sw))
PY
