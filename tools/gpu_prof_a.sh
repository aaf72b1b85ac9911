# round profiles, part A: configs 2 and 5 (rocprof kernel trace + FETCH_SIZE + WRITE_SIZE)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in 2 5; do bash profiles/collect.sh r02 $cfg || exit 1; echo "profiled c$cfg"; done
