# Kernel timeline of the RCCL tick transport (1 daemon, records to itself) with the
# tick thread's own statistics (post -> delivered, start() host time), then the
# copy-service sweep at the committed kernel (bench.py to 16 MiB) as a check.
set -o pipefail
OUT=${OUT:-gpurun_out/tickprof2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o tick -- python3 -u tools/ctrl_probe.py --variants rccl_stats --repeat 1 --out $OUT/ctrl_probe.json > $OUT/log.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ctrl_probe.py --variants rccl_stats,rccl_stats_nowait --repeat 2 --out $OUT/ctrl_probe_noprof.json > $OUT/log2.txt 2>&1 &&
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --max-bytes 16777216 --no-optim-extra --no-ctrl-extra --json-out $OUT/bench16m.json > $OUT/bench16m.log 2>&1
rc=$?; tail -3 $OUT/log.txt; grep -h "tick_stats" -A2 $OUT/ctrl_probe*.json | head -20; find $OUT -name "*kernel_trace.csv" | head; exit $rc
