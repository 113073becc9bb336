# round 4 (z15): PMC passes over the 1-GPU headline step (flat layout, native iteration)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4z15; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$R/gpurun_out/r4z15/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/r4z15/p$i.log" 2>&1 || exit 1
done
