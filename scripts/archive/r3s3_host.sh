#!/bin/bash
# session 3: host-issue trims (cheap stream switch, cached views) -- GPU tests of the
# touched paths, then bench at the driver's shape, 300 steps, B = 10,000, 8 emulated peers
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bench_pipeline_gpu.py tests/test_tp_fused_gpu.py tests/test_train_quality_gpu.py > gpurun_out/h_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/h_pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 120 python bench.py "$@" > gpurun_out/h_$tag.log 2>&1 || exit $?; \
  python - "$tag" gpurun_out/h_$tag.log <<'PY'
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
run e8 --emulate-peers 8 --steps 100 --warmup 10 || exit $?
run asp8 --emulate-peers 8 --consistency asp --fixing-float 2 --algo sgd --steps 100 --warmup 10 || exit $?
