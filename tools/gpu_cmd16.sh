# stream-pass workgroup size probe
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new new+ACC_ST_NT=256 new+ACC_ST_NT=1024
