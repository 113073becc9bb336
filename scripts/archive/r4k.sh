# round 4 (k): tile-count probe + r4j (Darlin, e8 eager host issue, B=10k variants, W&D ring GEMM)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/archive/r4i.sh || exit $?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/archive/r4j.sh
