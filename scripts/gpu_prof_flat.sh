set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c3_reasm c3_reasm6; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flat_$c -o run --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 5 --no-e2e --no-cpu --no-verify --reasm-flat 1 > gpurun_out/prof_flat_$c.txt 2>&1 || exit 1
done
