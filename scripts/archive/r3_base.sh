#!/bin/bash
# round-3 check: new kernels' tests first, then 1-GPU benches, train sweep, kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_tploc_gpu.py tests/test_gpu_ops.py tests/test_tp_fused_gpu.py > gpurun_out/r3_pytest_tp.log 2>&1 || { tail -30 gpurun_out/r3_pytest_tp.log; exit 1; }
tail -2 gpurun_out/r3_pytest_tp.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/r3_b1.log 2>&1 || exit $?
tail -1 gpurun_out/r3_b1.log | cut -c1-400
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --minibatch 10000 > gpurun_out/r3_b1_10k.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 100 --warmup 20 --emulate-peers 8 > gpurun_out/r3_e8.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 50 --warmup 20 --algo sgd --emulate-peers 8 --consistency asp --fixing-float 2 > gpurun_out/r3_cfg4.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/train_check.py --steps 50 lr:ftrl lr:adagrad lr:sgd lr:sgd:max_delta=0.05 lr:sgd:alpha=0.001 lr:sgd:alpha=0.0001,l1=1.0 lr:sgd:grad_scale=0.001,alpha=1.0,l1=0.01,l2=0.001 lr:sgd:grad_scale=0.01,alpha=0.1,l1=0.1,l2=0.01 fm fm:emb_lr=0.05 fm:emb_lr=0.01 fm:emb_lr=0.01,lambda_v=1.0 fm:emb_lr=0.02,wide_alpha=0.05 > gpurun_out/r3_train.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/r3_prof.log 2>&1 || exit $?
