# round-4 close: the N>1 bench path rehearsed with 2 ranks on the box's one GPU (gloo gradients)
PFSGNN_BENCH_SAME_DEVICE=1 PFSGNN_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --alt-paths , > gpurun_out/r04an_2rank.log 2>&1
