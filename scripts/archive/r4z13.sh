# round 4 (z13): driver shape with 2 vs 3 preparation streams (the short-run fill bubble at step 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z13
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2 3; do
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/p2_$r.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --prep-streams 3 > $O/p3_$r.log 2>&1 || exit $?
done
PSAMD_STEP_EVENTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --prep-streams 3 > $O/ev_p3.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 300 --warmup 10 --prep-streams 3 > $O/p3_300.log 2>&1 || exit $?
