# Last check of a round: the RCCL tick tests, smoke, the driver's N=1 bench and
# the 4-rank shared-GPU rehearsal, each under its own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_ctrl_tick.py tests/test_gpu_service.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json > $OUT/bench_n1.log 2>&1 &&
timeout -k 10 400 env OCM_BENCH_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --max-bytes 268435456 --json-out $OUT/bench_share4.json > $OUT/share4.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; tail -2 $OUT/smoke.log; tail -c 300 $OUT/bench_n1.log; exit $rc
