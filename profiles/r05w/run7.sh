#!/bin/bash
# r05w (7): does the host NUMA node of the packing threads explain the
# process-to-process spread (6.6 vs 8.3 ms) of the chunked HashBatch?
# cgo_path pinned (taskset) to the GPU's node vs the other node, alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w11; mkdir -p $O
bus=$(python3 -c "import glob,os; print('')")
for f in /sys/devices/system/node/node*/cpulist; do echo "$f $(cat $f)"; done > $O/nodes.txt
for d in /sys/bus/pci/drivers/amdgpu/0000:*; do echo "$d $(cat $d/numa_node 2>/dev/null)"; done >> $O/nodes.txt 2>&1
n0=$(cat /sys/devices/system/node/node0/cpulist)
n1=$(cat /sys/devices/system/node/node1/cpulist 2>/dev/null || echo $n0)
for r in 1 2 3; do
  taskset -c $n0 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_node0.json 2>> $O/cgo.err || exit 1
  taskset -c $n1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_node1.json 2>> $O/cgo.err || exit 1
done
echo done
