# N=1 bench.py at the driver's settings, five runs back to back on one box:
# run-to-run spread of the headline value and of the small-op latencies.
set -o pipefail
OUT=${OUT:-gpurun_out/soak}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/run_$i.json > $OUT/run_$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get('OUT', 'gpurun_out/soak')
for f in sorted(glob.glob(out + '/run_*.json')):
    d = json.load(open(f)); sw = d['sweep']
    print(os.path.basename(f), d['value'], d['alloc_p50_us'], ' '.join(f"{int(s)>>10}K:{sw[s]['get_us']}/{sw[s]['put_us']}" for s in ('4096', '262144', '1048576', '1073741824')))
PY
