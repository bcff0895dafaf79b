# round 5: fp64 multi-rank bench rehearsal (gloo, 4 ranks on the one GPU), chunked-dual records with per-iteration
# PMC, the full-size window test
export TMPDIR=/tmp
D=gpurun_out/r05d; mkdir -p $D
PDHG_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --steps 3 --warmup 1 --no-probe > $D/gloo4_fp64.json 2> $D/gloo4_fp64.err || { echo "gloo4 failed rc=$?"; exit 1; }
echo gloo4 ok
B="python bench.py --no-cpu-baseline --no-reference-precision --steps 10 --warmup 3 --no-probe"
run() { local tag=$1; shift; timeout -k 10 400 $B "$@" > $D/$tag.json 2> $D/$tag.err || { echo "$tag failed rc=$?"; exit 1; }; echo "$tag ok"; }
run c3_k10_fp32 --config c3 --precision fp32 --rho-alp-iters 10
run c2_k10_fp64 --config c2 --precision fp64 --rho-alp-iters 10
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_fullsize.py > $D/fullsize.log 2>&1; echo fullsize rc=$?
