set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || exit 1
for cfg in c3w1 c3; do
  echo "== $cfg"
  timeout -k 10 200 python bench.py --no-pmc --no-cpu-baseline --config $cfg --steps 20 --warmup 3 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('it/s %.2f ms %.4f' % (d['value'], d['ms_per_step']), {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" || exit 1
done
