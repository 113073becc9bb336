#!/bin/bash
# session 3: native launch list for the 1-GPU fused step -- the GPU suite, smoke, then
# bench at the driver's shape, 300 steps, B = 10,000
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/p_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/p_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/p_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/p_smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 120 python bench.py "$@" > gpurun_out/p_$tag.log 2>&1 || exit $?; \
  python - "$tag" gpurun_out/p_$tag.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], round(r["ms_per_step"], 4), round(r["host_issue_ms_per_step"], 4), round(r["value"] / 1e6, 1), r["train"]["loss"] < 0.6931)
PY
}
for rep in 1 2; do
  run d20_$rep --steps 20 --warmup 5 || exit $?
  run d300_$rep --steps 300 --warmup 10 || exit $?
  run b10k_$rep --minibatch 10000 --steps 300 --warmup 10 || exit $?
done
