# merge tests + config-5 A/B of reply-major slot loops
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_merge_gpu.py tests/test_deps_merge_gpu.py tests/test_latest_gpu.py tests/test_json_gpu.py tests/test_shard_gpu.py tests/test_levelise_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
CFGS="5" STEPS=10 bash tools/gpu_abn.sh new prerm
