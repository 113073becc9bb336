#!/bin/bash
# round 6: the AUC epilogue's stripes two per round (tpf_step / tpf_pack_grads extra workgroup)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r6z; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "auc or fused_1gpu or rccl or kw27 or pull_ahead or overlapped" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'), round(d['train'].get('loss'),4), round(d['train'].get('auc'),4))")"; }
run b20 --steps 20 --warmup 5 || exit 1
run base100 --steps 100 --warmup 10 || exit 1
run e8 --steps 100 --warmup 10 --emulate-peers 8 || exit 1
run b20b --steps 20 --warmup 5 || exit 1
run e8b --steps 100 --warmup 10 --emulate-peers 8 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_e8 -o run -- python $R/bench.py --steps 100 --warmup 10 --emulate-peers 8 > $O/p_e8.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_e8/run_results.db 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_1 -o run -- python $R/bench.py --steps 100 --warmup 10 > $O/p_1.log 2>&1 || exit 6
python $R/scripts/kdist_db.py $O/p_1/run_results.db 6
