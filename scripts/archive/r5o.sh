cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5o; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4))"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tploc_gpu.py tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python benchmarks/prof_tile_phases.py > $O/tile_phases.log 2>&1 || exit 4; grep -v amdgpu.ids $O/tile_phases.log
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b1_$i.log 2>&1 || exit 3; j $O/b1_$i.log "1gpu-20"; done
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $O/b300.log 2>&1 || exit 3; j $O/b300.log "1gpu-300"
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams 3 > $O/b10k.log 2>&1 || exit 3; j $O/b10k.log "B10k"
echo rc=0
