# Round-3 GPU check: N=1 bench (driver config) with the PCIe streaming kernel
# and with the SDMA baseline, rocprofv3 kernel stats of the bench, the GPU
# suite, smoke. Every step has its own time limit; a fault, abort, segfault or
# time limit ends the script (no further GPU step), an ordinary test failure
# does not.
set -o pipefail
OUT=gpurun_out/r03
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if fatal $rc; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step bench_n1 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json
step bench_n1_sdma 300 env OCM_HOST_ENGINE=sdma python3 -u bench.py --steps 20 --warmup 5 --no-optim-extra --json-out $OUT/bench_n1_sdma.json
step rocprof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-optim-extra --no-characterize
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
tail -3 $OUT/pytest_gpu.log
