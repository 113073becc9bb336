# round 4 (p): hardware queues vs streams: emulated peers / 1 GPU with GPU_MAX_HW_QUEUES 4 / 8
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4p
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/e8_q$q.log 2>&1 || exit $?
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --prep-streams 2 > $O/e8_p2_q$q.log 2>&1 || exit $?
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_q$q.log 2>&1 || exit $?
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 20 --warmup 5 --prep-streams 3 > $O/b20_p3_q$q.log 2>&1 || exit $?
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --prep-streams 4 > $O/e8_p4_q8.log 2>&1 || exit $?
