# The copy service's re-post after an idle exit (fresh seq): the interleave test
# at both idle exits, three passes, then the whole service and runtime files.
set -o pipefail
OUT=${OUT:-gpurun_out/relaunch}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -q -k interleave --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/interleave_$i.log 2>&1 || { tail -30 $OUT/interleave_$i.log; exit 1; }
  tail -1 $OUT/interleave_$i.log
done
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_service.py tests/test_gpu_runtime.py tests/test_fuzz_transfers.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/files.log 2>&1 || { tail -30 $OUT/files.log; exit 1; }
tail -1 $OUT/files.log
