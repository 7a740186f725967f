# Round 4: small-op latency mode against the NUMA node of the service's pages.
set -o pipefail
OUT=${OUT:-gpurun_out/r04u}
mkdir -p $OUT
export TMPDIR=/tmp
(numactl --hardware || true) > $OUT/numa.txt 2>&1
timeout -k 10 600 python3 -u tools/numa_mode_probe.py --procs 12 --out $OUT/numa_mode.json > $OUT/numa_mode.log 2>&1
rc=$?; head -5 $OUT/numa.txt; cat $OUT/numa_mode.log | cut -c1-300; exit $rc
