# round 4 (z16): per-GPU device cost of the N-GPU step at N = 2 / 4 / 8 emulated peers (RCCL loopback), final tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z16
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python bench.py --steps 100 --warmup 10 > $O/e1.log 2>&1 || exit $?
for n in 2 4 8; do
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers $n > $O/e$n.log 2>&1 || exit $?
done
