# round 4 (q): r4o (probe, tpf/tploc tests, benches) then r4p (hardware queue A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/archive/r4o.sh || exit $?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/archive/r4p.sh
