# Kernel timeline of the RCCL tick transport under the control-plane probe
# (1 daemon, records to itself): seal / allgather kernel durations and gaps.
set -o pipefail
OUT=gpurun_out/tickprof
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o tick -- python3 -u tools/ctrl_probe.py --variants rccl_spec_ccd --repeat 1 --out $OUT/ctrl_probe.json > $OUT/log.txt 2>&1
rc=$?; tail -5 $OUT/log.txt; find $OUT -name "*.csv" | head; exit $rc
