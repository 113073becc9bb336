# round 4 (z11): 8 emulated peers: owner-apply partition count (2^lgP key ranges)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4z11
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="python bench.py --steps 100 --warmup 10 --emulate-peers 8"
for r in 1 2; do
timeout -k 10 200 $B > $O/base_$r.log 2>&1 || exit $?
PSAMD_APPLY_LGP=8 timeout -k 10 200 $B > $O/lgp8_$r.log 2>&1 || exit $?
PSAMD_APPLY_LGP=10 timeout -k 10 200 $B > $O/lgp10_$r.log 2>&1 || exit $?
PSAMD_APPLY_LGP=11 timeout -k 10 200 $B > $O/lgp11_$r.log 2>&1 || exit $?
done
