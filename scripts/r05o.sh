#!/bin/bash
# round 5: fused residual at ny = 8192 by default (fp32 too) -- slab / fused / config tests, then c4w50 records
set -o pipefail
mkdir -p gpurun_out/r05o
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 700 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_slab64.py tests/test_gpu_fused.py \
  tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "fused or c4 or 8192" \
  > gpurun_out/r05o/tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r05o/tests.log | head; tail -5 gpurun_out/r05o/tests.log; exit 1; }
tail -3 gpurun_out/r05o/tests.log
for P in fp32 fp64; do
  timeout -k 10 400 python -u bench.py --config c4w50 --precision $P --steps 5 --warmup 2 --no-cpu-baseline \
    --no-probe --no-reference-precision > gpurun_out/r05o/c4w50_$P.json 2> gpurun_out/r05o/c4w50_$P.err || { tail -5 gpurun_out/r05o/c4w50_$P.err; exit 1; }
done
for P in fp32 fp64; do python - $P <<'P'
import json,sys
d=json.loads(open('gpurun_out/r05o/c4w50_%s.json'%sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d['ms_per_step'],2), {n:(round(v['avg_ms'],2), round((v.get('pmc_bytes_per_launch') or 0)/v['bytes_per_launch'],2)) for n,v in d['kernels'].items()})
P
done
