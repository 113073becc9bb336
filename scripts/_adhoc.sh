cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2 3; do for v in b1 b8; do
cp alt_so/_hipops_$v.so parameter_server_amd/_hipops.so
timeout -k 10 240 python bench.py --steps 300 --warmup 10 > gpurun_out/ab_${v}_$i.log 2>&1; echo "$v rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$i.log
done; done
