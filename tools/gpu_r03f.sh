# Round-3 validation at current code: N=1 bench (driver config), rocprofv3
# kernel stats of the bench, the 4-rank shared-GPU rehearsal of the N>1 path,
# the GPU suite, smoke. A fault, abort, segfault or time limit ends the script.
set -o pipefail
OUT=${OUT:-gpurun_out/r03f}
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
step rocprof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-characterize
step share4 400 env OCM_BENCH_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --max-bytes 268435456 --json-out $OUT/bench_share4.json
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
tail -3 $OUT/pytest_gpu.log
