# Round 4: the 8-rank one-GPU rehearsal with HIP lanes and with no lone lead (the
# tails after idle gaps under 16 processes), then the N=1 bench under rocprofv3.
set -o pipefail
mkdir -p gpurun_out/s8hip gpurun_out/s8lone0 gpurun_out/prof_r04
export TMPDIR=/tmp
OUT=gpurun_out/s8hip PORT=29561 OCM_SERVICE_QUEUE=hip timeout -k 10 400 bash tools/gpu_share8.sh &&
OUT=gpurun_out/s8lone0 PORT=29571 OCM_SERVICE_LONE_US=0 timeout -k 10 400 bash tools/gpu_share8.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04 -o bench -- python3 -u bench.py --steps 5 --warmup 2 --json-out gpurun_out/prof_r04/bench.json > gpurun_out/prof_r04/bench.log 2>&1
rc=$?; find gpurun_out/prof_r04 -name "*kernel_stats.csv" | head -3; exit $rc
