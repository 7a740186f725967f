# Round-3 GPU check c: kernel numerics (write-through register kernel), the
# control-plane probe with longer spin windows, and the N=4 one-GPU rehearsal
# (autotune with the write-through and push candidates).
set -o pipefail
OUT=gpurun_out/r03c
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
step kernels 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_ctrl_tick.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
step ctrl 300 python3 -u tools/ctrl_probe.py --variants rccl_spec_ccd,rccl_spec_ccd_spin300 --repeat 4 --out $OUT/ctrl_probe.json
step share4 400 env OCM_BENCH_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --max-bytes 268435456 --json-out $OUT/bench_share4.json
tail -2 $OUT/kernels.log
