# session check 11: radix sort with per-digit column scans: broad GPU tests, then A/B on configs 2, 3, 4
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new prers || exit 1
CFGS="4" STEPS=5 bash tools/gpu_abn.sh new prers
