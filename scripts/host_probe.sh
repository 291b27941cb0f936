#!/bin/bash
# What the GPU box's host offers the CPU baselines: cores, affinity, cgroup quota, model.
echo "nproc=$(nproc) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo none)"
python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"
grep -m1 "model name" /proc/cpuinfo
