# Small-op latency vs where the app runs: bench.py's host-tier sweep to 1 MiB with
# the app on the GPU's NUMA node, on the other node, unpinned, and with OCM_PIN=1
# (the library pins the app thread next to the GPU), interleaved, 2 rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/numa}
mkdir -p $OUT
GN=$(cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -1)
echo "gpu numa_node=$GN nodes=$(ls -d /sys/devices/system/node/node* | wc -l)"
N0=$(cat /sys/devices/system/node/node0/cpulist); N1=$(cat /sys/devices/system/node/node1/cpulist 2>/dev/null || echo $N0)
echo "node0=$N0 node1=$N1"
run() { timeout -k 10 200 "$@" python3 -u bench.py --steps 20 --warmup 3 --max-bytes 1048576 --no-optim-extra --no-ctrl-extra --json-out $OUT/$NAME.json > $OUT/$NAME.log 2>&1; }
for i in 1 2; do
  NAME=node0_$i run taskset -c $N0 || exit $?
  NAME=node1_$i run taskset -c $N1 || exit $?
  NAME=free_$i run env || exit $?
  NAME=pin_$i run env OCM_PIN=1 || exit $?
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get('OUT', 'gpurun_out/numa')
for f in sorted(glob.glob(out + '/*.json')):
    d = json.load(open(f)); sw = d['sweep']
    print(os.path.basename(f), 'alloc', d.get('alloc_p50_us'), ' '.join(f"{int(s)>>10}K:{sw[s]['get_us']}/{sw[s]['put_us']}" for s in sw))
PY
