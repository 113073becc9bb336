cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TESTS="tests/test_sharded_kv.py tests/test_embedding_checkpoint.py" BENCHES="1 e8 --localize=part e8asp" bash scripts/gpu_quick.sh || exit 1
timeout -k 10 100 python -m parameter_server_amd.app.hello_world_gpu > gpurun_out/hello_gpu.log 2>&1; echo hello rc=$?; tail -6 gpurun_out/hello_gpu.log
