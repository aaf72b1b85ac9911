# round-2 session check: KeyDeps / levelise / merge GPU tests, then same-box timing of library variants
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_keydeps_gpu.py tests/test_keydeps_mixed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 300 python -u -m pytest tests/test_levelise_gpu.py tests/test_merge_gpu.py tests/test_deps_merge_gpu.py tests/test_rangedeps_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new base new+serial || exit 1
CFGS="5 4" STEPS=5 bash tools/gpu_abn.sh new base
