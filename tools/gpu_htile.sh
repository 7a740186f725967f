# Host-tier tile size A/B for direct gangs (service probe, host tier).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/svc_probe.py --tiers host --configs default,htile12,htile13,htile14,htile13p --repeat 2 --out gpurun_out/svc_htile.json > gpurun_out/svc_htile.log 2>&1
