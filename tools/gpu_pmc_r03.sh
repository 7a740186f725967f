# PMC passes (one counter group per run, kernel trace only) over the data-plane
# kernels: bytes fetched / written per dispatch for the copy service, the PCIe
# streaming kernel and the host-tier fused Adam.
set -o pipefail
OUT=gpurun_out/pmc_r03
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o fetch -- python3 tools/pmc_service.py > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o write -- python3 tools/pmc_service.py > $OUT/write.log 2>&1
rc=$?; tail -3 $OUT/fetch.log; tail -3 $OUT/write.log; find $OUT -name "*.csv" | head; exit $rc
