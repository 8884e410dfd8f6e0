#!/bin/bash
# Host-topology probe for the GPU box (NUMA, CXL, memory); run under gpurun.
mkdir -p gpurun_out
{
  echo "== nproc/meminfo"; nproc; head -5 /proc/meminfo
  echo "== numa nodes"; ls /sys/devices/system/node/ | grep node
  for n in /sys/devices/system/node/node*; do echo "$n cpus=$(cat $n/cpulist) mem=$(grep MemTotal $n/meminfo)"; done
  echo "== cxl"; ls /sys/bus/cxl/devices 2>&1 | head
  echo "== hugepages"; cat /proc/sys/vm/nr_hugepages; grep -i huge /proc/meminfo
  echo "== thp"; cat /sys/kernel/mm/transparent_hugepage/enabled
  echo "== ulimit -l"; ulimit -l
  echo "== rocm-smi"; timeout 60 rocm-smi --showtopo 2>&1 | head -40
  echo "== gpu numa"; for d in /sys/class/drm/card*/device/numa_node; do echo "$d $(cat $d)"; done
  echo "== userfaultfd"; cat /proc/sys/vm/unprivileged_userfaultfd 2>&1
} > gpurun_out/probe_host.txt 2>&1
mkdir -p build
hipcc --offload-arch=gfx950 -O3 tools/probe_box.hip -o build/probe_box && timeout -k 10 300 ./build/probe_box 8192 > gpurun_out/probe_gpu.txt 2>&1
rc=$?
cat gpurun_out/probe_host.txt gpurun_out/probe_gpu.txt
exit $rc
