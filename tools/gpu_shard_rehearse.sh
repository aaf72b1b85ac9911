# N > 1 bench path on a one-GPU box: N ranks on GPU 0 over gloo (everything but RCCL).
#   bash tools/gpu_shard_rehearse.sh [N=8] [config=3] [scale=0.05]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=${1:-8}; CFG=${2:-3}; SCALE=${3:-0.05}
export ACC_BENCH_REHEARSE=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --config $CFG --gpus $N --steps 3 --warmup 1 --scale $SCALE > gpurun_out/rehearse_n${N}_c${CFG}.log 2>&1
rc=$?
tail -3 gpurun_out/rehearse_n${N}_c${CFG}.log
exit $rc
