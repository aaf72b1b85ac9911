# session check 4: full GPU tests + bench lines (gpu_round.sh), then timing variants
cd $GRAFT_REPO_ROOT && bash tools/gpu_round.sh r02 || exit 1
CFGS="5" STEPS=10 bash tools/gpu_abn.sh new lvg32 lvg64 lvp8 || exit 1
CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new prehoist
