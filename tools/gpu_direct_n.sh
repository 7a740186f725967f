# Direct gang pollers (OCM_SERVICE_DIRECT: workgroups that poll the host gang
# record themselves; gangs up to that width skip the relay): 16 (default) vs 8
# vs 4, host-tier sweep to 4 MiB, interleaved, 3 rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/directn}
mkdir -p $OUT
for i in 1 2 3; do
  for d in 16 8 4; do
    timeout -k 10 200 env OCM_SERVICE_DIRECT=$d python3 -u bench.py --steps 10 --warmup 3 --max-bytes 4194304 --no-optim-extra --no-ctrl-extra --json-out $OUT/d${d}_$i.json > $OUT/d${d}_$i.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get('OUT', 'gpurun_out/directn')
for f in sorted(glob.glob(out + '/*.json')):
    d = json.load(open(f)); sw = d['sweep']
    print(os.path.basename(f), ' '.join(f"{int(s)>>10}K:{sw[s]['get_us']}/{sw[s]['put_us']}" for s in sw))
PY
