# levelise group-size probe (8 lanes per position)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
CFGS="5" STEPS=10 bash tools/gpu_abn.sh new lvg8
