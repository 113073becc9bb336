#!/bin/bash
# round 6: PMC passes (SQ counters) over the tail-filtered 1-GPU step and the 8-peer step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=gpurun_out/r6ze; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_tpf_gpu.py tests/test_bench_pipeline_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "tail or kw27 or kw28 or kw29" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -5 $O/$n.log; return 1; }; echo "$n: $(grep '^{' $O/$n.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],4))")"; }
run tail1 --steps 100 --warmup 10 --tail-freq 1 || exit 1
run base100 --steps 100 --warmup 10 || exit 1
run tail1b --steps 100 --warmup 10 --tail-freq 1 || exit 1
cd /tmp
i=0
for args in "--tail-freq 1" "--emulate-peers 8"; do
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set -d "$R/$O/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 $args > "$R/$O/p$i.log" 2>&1 || exit 1
    echo "pass $i ($args) ok"
  done
done
cd $R
python scripts/pmc_sum.py $O psamd > $O/summary.txt; cat $O/summary.txt | cut -c1-400
