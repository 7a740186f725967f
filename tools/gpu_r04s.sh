# Round 4: GPU read latency of host memory by allocation kind (three runs).
set -o pipefail
OUT=${OUT:-gpurun_out/r04s}
mkdir -p $OUT
timeout -k 10 60 build/bin/host_mem_latency_probe > $OUT/hostmem1.json 2>&1 &&
timeout -k 10 60 build/bin/host_mem_latency_probe > $OUT/hostmem2.json 2>&1 &&
timeout -k 10 60 build/bin/host_mem_latency_probe > $OUT/hostmem3.json 2>&1
rc=$?; cat $OUT/hostmem*.json; exit $rc
