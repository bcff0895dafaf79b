set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02z
mkdir -p $OUT
PDHG_UPD_PF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread -x > $OUT/t.log 2>&1; echo "t rc=$?"
bash scripts/sweep_env.sh PDHG_UPD_PF "0 1 0 1 0 1" --config c3 --steps 6 --warmup 1 --no-probe > $OUT/sweep.log 2>&1 || exit 1
echo all-done
