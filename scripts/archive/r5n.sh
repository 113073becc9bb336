cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5n; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python benchmarks/prof_tile_phases.py > $O/tile_phases.log 2>&1; rc=$?; cat $O/tile_phases.log | grep -v amdgpu.ids; exit $rc
