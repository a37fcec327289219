# one GPU session (round 4): the GPU suite, smoke, bench lines of the main configs, kernel traces of
# C1 (graph replay and launched one by one) / C2 / C2 slot ring, a short interleaved A/B against the
# round-3 stream kernels (picotcp_amd/ab/libpicocsum_r03.so), then the PMC passes of the round
# (scripts/gpu_pmc_round.sh).  Every GPU step under its own time limit; the first failure ends it.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r04a}
mkdir -p $O
cd $R
# provenance: the library rebuilt from source on the box (make -B), build() then loads it
timeout -k 10 600 make -s -B -j16 -C picotcp_amd/csrc > $O/build_$TAG.log 2>&1
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build(); print('build ok')" >> $O/build_$TAG.log 2>&1
echo "build ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1
echo "smoke ok"
timeout -k 10 400 python bench.py > $O/bench_c1_$TAG.json 2> $O/bench_c1_$TAG.err
echo "bench c1 ok"
for c in c2 c2slot c2ethmix c2v6 c2eth c2nat c2tx; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
for c in c1 c2 c2slot; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 100 --warmup 10 --no-cpu --no-e2e --no-verify > $O/prof_${c}_$TAG.log 2>&1
  echo "trace $c ok"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1ng_$TAG -o run --output-format csv -- python3 $R/bench.py --no-graph --no-cpu --no-e2e --no-verify > $O/prof_c1ng_$TAG.log 2>&1
echo "trace c1 no-graph ok"
cd $R
A=r03 ROUNDS=2 CFGS="c2 c2eth c2ethmix c2v6" bash scripts/gpu_ab.sh r03_$TAG
echo "ab r03 ok"
bash scripts/gpu_pmc_round.sh $TAG
echo "pmc ok"
