set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02v
mkdir -p $OUT
PDHG_DUAL_PD=2 PDHG_DBG=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_slab.py -q -rf --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; echo "t rc=$?"
for cfg in "1 0" "2 0" "1 16" "2 16" "1 0" "2 0" "1 16" "2 16"; do
  set -- $cfg
  echo "== DUAL_PD=$1 DBG=$2" >> $OUT/sweep.log
  PDHG_DUAL_PD=$1 PDHG_DBG=$2 timeout -k 10 300 python bench.py --config c3 --steps 6 --warmup 1 --no-probe --no-pmc --no-cpu-baseline > $OUT/b.json 2>>$OUT/b.err || exit 1
  python -c "
import json,sys
d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('it/s %.3f' % d['value'], {k: round(v['avg_ms'],2) for k,v in d['kernels'].items()})" >> $OUT/sweep.log
done
echo all-done
