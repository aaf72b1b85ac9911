# round profiles, part B: configs 3 and 4
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in 3 4; do bash profiles/collect.sh r02 $cfg || exit 1; echo "profiled c$cfg"; done
