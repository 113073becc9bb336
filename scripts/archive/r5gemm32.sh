cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5gemm32; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 300 python benchmarks/bench_gemm256.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
python - <<PY
import json
for l in open('$O/bench.log'):
    if l.startswith('{'):
        d=json.loads(l)
        print(d.get('shape'), {k:round(v) for k,v in d.items() if k.endswith('tflops')}, d.get('max_rel_err_vs_fp32', [None])[-1] if 'max_rel_err_vs_fp32' in d else '')
PY
