# medium KeyDeps tier on 512-thread workgroups: tests + A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_keydeps_gpu.py tests/test_keydeps_mixed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new premed
