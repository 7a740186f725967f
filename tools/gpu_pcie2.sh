set -o pipefail
mkdir -p gpurun_out/pcie2
P=./build/tools/pcie_stream_probe
timeout -k 10 240 $P 268435456 3 put 16,32,48,64,96,128,192,256 "la0/,la2/" > gpurun_out/pcie2/put_256m.json 2> gpurun_out/pcie2/put.err &&
timeout -k 10 200 $P 268435456 3 get 32,64,96,128,192,256 "sa0,sa2" > gpurun_out/pcie2/get_256m.json 2> gpurun_out/pcie2/get.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pcie2/prof -o blit -- $GRAFT_REPO_ROOT/build/tools/pcie_stream_probe 268435456 2 both 128 zzz > $GRAFT_REPO_ROOT/gpurun_out/pcie2/blit.json 2> $GRAFT_REPO_ROOT/gpurun_out/pcie2/blit.err
echo rc=$?
