set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
A=wpb1 ROUNDS=2 CFGS="c2 c2v6 c2eth" bash scripts/gpu_ab.sh wpb1_w1
A=wpb2 ROUNDS=2 CFGS="c2 c2v6 c2eth" bash scripts/gpu_ab.sh wpb2_w1
