# Host page size vs PCIe streaming: the box's THP settings, then the PCIe kernel
# shapes the library uses (8 KiB tiles: u2; 128 workgroups) on the memfd slab and
# on anonymous THP memory, both directions, 1 GiB.
set -o pipefail
OUT=gpurun_out/thp
mkdir -p $OUT
cat /sys/kernel/mm/transparent_hugepage/shmem_enabled /sys/kernel/mm/transparent_hugepage/enabled > $OUT/thp.txt 2>&1
P=./build/tools/pcie_stream_probe
timeout -k 10 200 $P 1073741824 3 both 128 "0/u2/la2/sa0,0/u2/la2/sa16" > $OUT/memfd.json 2> $OUT/memfd.err &&
timeout -k 10 200 $P 1073741824 3 both 128 "0/u2/la2/sa0,0/u2/la2/sa16" anonhuge > $OUT/anonhuge.json 2> $OUT/anonhuge.err &&
grep -i -E "AnonHuge|ShmemHuge" /proc/meminfo >> $OUT/thp.txt
rc=$?; cat $OUT/thp.txt; cat $OUT/memfd.json $OUT/anonhuge.json; exit $rc
