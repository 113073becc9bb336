cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
for pr in 0 -1; do
PSAMD_PREP_PRIORITY=$pr timeout -k 10 240 python bench.py --steps 100 --warmup 10 --emulate-peers 8 --emulate-backend nccl > gpurun_out/e8n_p$pr.log 2>&1; echo "nccl prio $pr rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8n_p$pr.log
PSAMD_PREP_PRIORITY=$pr timeout -k 10 240 python bench.py --steps 100 --warmup 10 --emulate-peers 8 > gpurun_out/e8_p$pr.log 2>&1; echo "copy prio $pr rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/e8_p$pr.log
done
cd /tmp && PSAMD_PREP_PRIORITY=-1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/profe8n2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 10 --emulate-peers 8 --emulate-backend nccl > "$GRAFT_REPO_ROOT/gpurun_out/profe8n2.log" 2>&1; echo prof rc=$?
