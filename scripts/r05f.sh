# round 5: half-real LDS-DMA x transform (C4's nx = 8192): parity against the warp-specialised kernel, slabs,
# fixtures; c4w50 A/B
export TMPDIR=/tmp
D=gpurun_out/r05f; mkdir -p $D
B="python bench.py --no-cpu-baseline --no-reference-precision --steps 6 --warmup 2 --no-probe --no-pmc --config c4w50 --precision fp32"
PDHG_XT_DMA_HR=1 timeout -k 10 300 $B > $D/c4w50_dmahr.json 2> $D/c4w50_dmahr.err || exit 1
PDHG_XT_DMA_HR=0 timeout -k 10 300 $B > $D/c4w50_ws.json 2> $D/c4w50_ws.err || exit 1
echo bench ok
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py \
  tests/test_gpu_slab.py -k "halfreal or 8192" \
  > $D/t.log 2>&1; echo tests rc=$?
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py -k "c4" \
  > $D/t2.log 2>&1; echo decomp rc=$?
