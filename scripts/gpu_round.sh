#!/bin/bash
# One round's measurement session (bench lines + rocprofv3 kernel traces), every GPU step under its
# own time limit; any failure ends the script.  Outputs gpurun_out/bench_<cfg>_$TAG.json and
# gpurun_out/prof_<cfg>_$TAG/ (run_kernel_stats.csv); tools/record_profiles.py copies them into
# profiles/<round>/.  PMC passes: scripts/gpu_pmc_round.sh.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_c1_$TAG.json 2> $O/bench_c1_$TAG.err
echo "bench c1 ok"
for c in ${BENCHES:-c2 c2slot c2tx c2tx_nw c2nat c2v6 c2eth c2ethmix c3_reasm c3_reasm6}; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
for c in ${TRACES:-c1 c2 c2slot c2tx c2nat c2v6 c2eth c2ethmix c3_reasm c3_reasm6}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 100 --warmup 10 --no-cpu --no-e2e --no-verify > $O/prof_${c}_$TAG.log 2>&1
  echo "trace $c ok"
done
# C1 launched one by one (no graph): the same comparison without the graph replay
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1ng_$TAG -o run --output-format csv -- python3 $R/bench.py --no-graph --no-cpu --no-e2e --no-verify > $O/prof_c1ng_$TAG.log 2>&1
echo "trace c1 no-graph ok"
