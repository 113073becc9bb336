cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z6; mkdir -p $O
export PYTHONUNBUFFERED=1
for n in 2 3; do for i in 1 2; do
  PSAMD_STEP_EVENTS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --prep-streams $n > $O/n${n}_$i.log 2>&1 || exit 3
  echo "n=$n"; grep step_events_ms $O/n${n}_$i.log | cut -c1-400
done; done
