cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5q; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_gemm256.py > $O/bench.log 2>&1; rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/r5q/bench.log"):
    if not l.startswith("{"): continue
    d=json.loads(l)
    print(d["shape"], {k: round(v) for k, v in d.items() if k.endswith("tflops")}, d.get("max_rel_err_vs_fp32"))
PY
exit $rc
