# Copy-service gang width (OCM_SERVICE_BLOCKS) and HBM bound under the direct-record protocol, both tiers.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u tools/svc_probe.py --tiers host,hbm --configs default,blocks128,blocks256,blocks128_max64,blocks256_max64 --repeat 2 --out gpurun_out/svc_blocks.json > gpurun_out/svc_blocks.log 2>&1
