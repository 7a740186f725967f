# Round-3 GPU check b: the GPU suite (push get, pool release), then the N=4
# one-GPU rehearsal with autotune (push candidates included). Every step has a
# time limit; a fault, abort, segfault or time limit ends the script.
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
step() {
    local name=$1 secs=$2
    shift 2
    timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if fatal $rc; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
step share4 400 env OCM_BENCH_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --max-bytes 268435456 --json-out $OUT/bench_share4.json
tail -3 $OUT/pytest_gpu.log
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
