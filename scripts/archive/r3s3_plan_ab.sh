#!/bin/bash
# session 3: native step plan on / off (PSAMD_STEP_PLAN), interleaved on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_tp_fused_gpu.py > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 120 python bench.py "$@" > gpurun_out/ab_$tag.log 2>&1 || exit $?; \
  python - "$tag" gpurun_out/ab_$tag.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], round(r["ms_per_step"], 4), round(r["host_issue_ms_per_step"], 4), round(r["value"] / 1e6, 1), r["train"]["loss"] < 0.6931)
PY
}
for rep in 1 2 3; do
  PSAMD_STEP_PLAN=1 run plan1_b10k_$rep --minibatch 10000 --steps 500 --warmup 10 || exit $?
  PSAMD_STEP_PLAN=0 run plan0_b10k_$rep --minibatch 10000 --steps 500 --warmup 10 || exit $?
  PSAMD_STEP_PLAN=1 run plan1_d20_$rep --steps 20 --warmup 5 || exit $?
  PSAMD_STEP_PLAN=0 run plan0_d20_$rep --steps 20 --warmup 5 || exit $?
done
