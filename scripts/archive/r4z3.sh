# round 4 (z3): 8 emulated peers (RCCL loopback): where the exchange half runs, how far ahead, queues
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z3
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="python bench.py --steps 100 --warmup 10 --emulate-peers 8"
timeout -k 10 200 $B > $O/base.log 2>&1 || exit $?
PSAMD_XCHG_STREAM=own timeout -k 10 200 $B --prep-streams 2 > $O/own_p2.log 2>&1 || exit $?
PSAMD_XCHG_STREAM=own timeout -k 10 200 $B > $O/own_p3.log 2>&1 || exit $?
PSAMD_XD=3 timeout -k 10 200 $B > $O/xd3.log 2>&1 || exit $?
PSAMD_XD=1 timeout -k 10 200 $B > $O/xd1.log 2>&1 || exit $?
timeout -k 10 200 $B --prep-streams 2 > $O/p2.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B > $O/hwq8.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 PSAMD_XCHG_STREAM=own timeout -k 10 200 $B > $O/hwq8_own.log 2>&1 || exit $?
timeout -k 10 200 $B > $O/base2.log 2>&1 || exit $?
bash scripts/r4z4.sh
