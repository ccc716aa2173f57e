#!/bin/bash
# What the GPU box offers the CPU baseline: CPU model, cores, affinity, cgroup quota,
# and the PMC counters rocprofv3 can collect on this GPU.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
{
  echo "nproc: $(nproc)"
  python3 -c 'import os; print("affinity:", len(os.sched_getaffinity(0)), "cpu_count:", os.cpu_count())'
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"
  grep -m1 "model name" /proc/cpuinfo
  lscpu 2>/dev/null | head -20
} > "$R/gpurun_out/boxinfo.log" 2>&1
timeout -k 10 120 rocprofv3 --list-avail > "$R/gpurun_out/counters.txt" 2>&1
exit 0
