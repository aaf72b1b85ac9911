# N > 1 bench path on a one-GPU box: 2 ranks on GPU 0 over gloo (everything but RCCL), 1/4 scale
set -o pipefail
cd $GRAFT_REPO_ROOT
export ACC_BENCH_REHEARSE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --steps 3 --warmup 1 --scale 0.25 > gpurun_out/rehearse.log 2>&1
rc=$?
tail -5 gpurun_out/rehearse.log
exit $rc
