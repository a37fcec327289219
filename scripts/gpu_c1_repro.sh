#!/bin/bash
# C1 roofline reproducibility: the default bench line and the rocprofv3
# kernel trace OF THE SAME PROCESS (its own bench line is kept in the log), graph replay and
# --no-graph, plus the host CPU share the box grants (cgroup quota).  Every GPU step has its own
# time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c1repro
TAG=${1:-run}
mkdir -p $O
cd $R
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max";
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'OMP', os.environ.get('OMP_NUM_THREADS'))"; } > $O/host_$TAG.txt
timeout -k 10 300 python bench.py > $O/bench_graph_$TAG.json 2> $O/bench_graph_$TAG.err
echo "bench graph ok"
timeout -k 10 300 python bench.py --no-graph --no-cpu --no-e2e > $O/bench_nograph_$TAG.json 2> $O/bench_nograph_$TAG.err
echo "bench nograph ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_graph_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu --no-e2e --no-verify > $O/prof_graph_$TAG.log 2>&1
echo "trace graph ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_nograph_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --no-graph --no-cpu --no-e2e --no-verify > $O/prof_nograph_$TAG.log 2>&1
echo "trace nograph ok"
