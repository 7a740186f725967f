# Round 4, first GPU pass: the copy-service roster fix. Service tests (with the
# CU hog), the 4-thread fuzz, the 4-rank shared-GPU rehearsal and the N=1 bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r04a}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1 &&
timeout -k 10 300 python3 -u tools/gpu_fuzz.py --seconds 45 --seed 41 --threads 4 --configs hbm,stripe,host,net --out $OUT/fuzz_t4.json > $OUT/fuzz_t4.log 2>&1 &&
timeout -k 10 400 env OCM_BENCH_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --max-bytes 268435456 --json-out $OUT/bench_share4.json > $OUT/share4.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json > $OUT/bench_n1.log 2>&1
rc=$?; tail -3 $OUT/pytest_service.log; tail -2 $OUT/fuzz_t4.log | cut -c1-400; grep -c "copy service failed" $OUT/*.log; tail -c 300 $OUT/bench_n1.log; exit $rc
