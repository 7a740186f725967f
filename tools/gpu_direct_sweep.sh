# Number of direct gang pollers (OCM_SERVICE_DIRECT), service probe on both tiers.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u tools/svc_probe.py --tiers host,hbm --configs default,direct8,direct12,direct24,direct32 --repeat 2 --out gpurun_out/svc_direct_sweep.json > gpurun_out/svc_direct_sweep.log 2>&1
