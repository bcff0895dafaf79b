set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_slab.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_slab.log 2>&1 || exit 1
timeout -k 10 300 python scripts/slab_local_bench.py tslab c3 8 3 > gpurun_out/slab8.json 2> gpurun_out/slab8.err || exit 1
export PDHG_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/b_n2.json 2> gpurun_out/b_n2.err || exit 1
