# Alloc-latency A/B on one box: bench.py's alloc phase with the app on each
# NUMA node in turn (its daemon stays pinned next to the GPU), with the
# shared-memory link and with the mailbox alone.
set -o pipefail
OUT=gpurun_out/alloc_ab2
mkdir -p $OUT
for node in 0 1; do
  cpus=$(cat /sys/devices/system/node/node$node/cpulist)
  for link in 1 0; do
    for i in 1 2; do
      timeout -k 10 200 env OCM_SHM_LINK=$link taskset -c $cpus python3 -u bench.py --steps 1 --warmup 0 --max-bytes 1048576 --no-optim-extra --no-characterize --json-out $OUT/n${node}_link${link}_$i.json > $OUT/n${node}_link${link}_$i.log 2>&1 || exit $?
    done
  done
done
cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -3
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d.get('alloc_p50_us'), d.get('alloc_p99_us'), d.get('local_alloc_p50_us'), d.get('free_p50_us'))"; done
