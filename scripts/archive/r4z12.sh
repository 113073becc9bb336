# round 4 (z12): per-step GPU times of the driver-shape run (fill / drain of short runs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z12
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2 3; do
PSAMD_STEP_EVENTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/ev_$r.log 2>&1 || exit $?
done
