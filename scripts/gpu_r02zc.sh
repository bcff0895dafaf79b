set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02zc
mkdir -p $OUT
L=pdhg-optimal-control_amd/pdhg_amd
cp $L/libpdhg.so $OUT/../libpdhg_default.so.bak
run() {
  timeout -k 10 300 python bench.py --config c3 --steps 6 --warmup 1 --no-probe --no-pmc --no-cpu-baseline > $OUT/b.json 2>>$OUT/b.err || return 1
  python -c "
import json
d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('it/s %.3f' % d['value'], {k: round(v['avg_ms'],2) for k,v in d['kernels'].items()})" >> $OUT/sweep.log
}
for v in default upd default upd; do
  echo "== $v" >> $OUT/sweep.log
  if [ $v = upd ]; then cp $L/libpdhg_upd.so $L/libpdhg.so; else cp $OUT/../libpdhg_default.so.bak $L/libpdhg.so; fi
  touch $L/libpdhg.so
  run || exit 1
done
cp $L/libpdhg_upd.so $L/libpdhg.so && touch $L/libpdhg.so
timeout -k 10 450 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; echo "t rc=$?"
rm -f $OUT/../libpdhg_default.so.bak
echo all-done
