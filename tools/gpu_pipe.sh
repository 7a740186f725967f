# Pipelined host polls of the copy service (PIPE2 = 32, PIPE4 = 64 protocol bits
# on top of the default 15): the service GPU tests under PIPE4, then bench.py's
# sweep up to 16 MiB (the service's host-tier range), interleaved.
set -o pipefail
OUT=${OUT:-gpurun_out/pipe}
mkdir -p $OUT
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 env OCM_SERVICE_PROTO=79 python3 -u -m pytest tests/test_gpu_service.py tests/test_gpu_runtime.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  for p in ${PROTOS:-15 47 79}; do
    timeout -k 10 200 env OCM_SERVICE_PROTO=$p python3 -u bench.py --steps 10 --warmup 3 --max-bytes 16777216 --no-optim-extra --no-ctrl-extra --json-out $OUT/p${p}_$i.json > $OUT/p${p}_$i.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get('OUT', 'gpurun_out/pipe')
for f in sorted(glob.glob(out + '/p*.json')):
    d = json.load(open(f)); sw = d['sweep']
    print(f.split('/')[-1], ' '.join(f"{int(s)>>10}K:{sw[s]['get_us']}/{sw[s]['put_us']}" for s in sw))
PY
