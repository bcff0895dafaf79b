# round 5: fp64 x kernel at nx 512 / 1024 / 2048 vs generic + oracle, fp64 slabs on C3's whole plane, dual-multi time
# chunks, marching counts under the dual shortcuts' toggles
export TMPDIR=/tmp
D=gpurun_out/r05e; mkdir -p $D
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_xt64.py \
  tests/test_gpu_slab64.py tests/test_gpu_dual_multi.py "tests/test_gpu_parity.py::test_marching_window_counts_fp64" \
  > $D/t.log 2>&1; echo tests rc=$?
