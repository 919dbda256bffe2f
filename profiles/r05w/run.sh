#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w; mkdir -p $O
{
echo "nproc $(nproc)"
cat /proc/self/cgroup
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/cpu.stat; do echo "== $f"; cat $f 2>&1; done
python3 -c 'import os; print("sched_getaffinity", len(os.sched_getaffinity(0)))'
} > $O/cgroup_before.txt 2>&1
for r in 1 2 3; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo15.json 2>> $O/cgo.err || exit 1
  cat /sys/fs/cgroup/cpu.stat >> $O/cpustat_15.txt 2>&1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 11 7 32 nt >> $O/cgo11.json 2>> $O/cgo.err || exit 1
  cat /sys/fs/cgroup/cpu.stat >> $O/cpustat_11.txt 2>&1
done
echo done
