#!/bin/bash
# round 6: PMC passes (SQ counters) over the tail-filtered 1-GPU step and the 8-peer step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=gpurun_out/r6ze; mkdir -p $O
export TMPDIR=/tmp
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
