mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dist.log 2>&1; rc=$?; tail -8 gpurun_out/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --rows-per-gpu 2e9 > gpurun_out/b2.json 2> gpurun_out/b2.err; rc=$?; cat gpurun_out/b2.json; tail -3 gpurun_out/b2.err; exit $rc
