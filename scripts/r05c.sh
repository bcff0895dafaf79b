# round 5: per-GPU fp64 lines (C2 with the new nx = 2048 x kernel, C3 / C4 per-GPU slabs' shapes), chunked-dual
# records with pass bytes, the full-size window test
export TMPDIR=/tmp
D=gpurun_out/r05c; mkdir -p $D
B="python bench.py --no-cpu-baseline --no-reference-precision --steps 10 --warmup 3"
run() { local tag=$1; shift; timeout -k 10 400 $B "$@" > $D/$tag.json 2> $D/$tag.err || { echo "$tag failed rc=$?"; exit 1; }; echo "$tag ok"; }
run c2_fp64 --config c2 --precision fp64
run c3w25_fp64 --config c3w25 --precision fp64
run c4w50_fp64 --config c4w50 --precision fp64 --no-probe
run c3_k10_fp32 --config c3 --precision fp32 --rho-alp-iters 10 --no-probe
run c2_k10_fp64 --config c2 --precision fp64 --rho-alp-iters 10 --no-probe
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_fullsize.py > $D/fullsize.log 2>&1; echo fullsize rc=$?
