set -u
mkdir -p gpurun_out/exp5
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
   bench.py --gpus 2 --config lfr100k --steps 2 --warmup 1 --dist-backend gloo > gpurun_out/exp5/gloo2.json 2> gpurun_out/exp5/gloo2.err || exit $?
echo gloo2 done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
   bench.py --gpus 2 --config lfr100k --steps 2 --warmup 1 > gpurun_out/exp5/nccl2.json 2> gpurun_out/exp5/nccl2.err
echo "nccl2 rc=$?"
