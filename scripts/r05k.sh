#!/bin/bash
# round 5: fp64 fused residual at ny = 8192 (C4) -- tests, then the c4w50 fp64 per-GPU line
set -o pipefail
mkdir -p gpurun_out/r05k
export PYTHONPATH=$PWD/pdhg-optimal-control_amd:$PWD/oracle:$PWD/tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_configs.py -x -v --timeout 300 \
  --timeout-method thread -k "fp64 and not (fused_fp64_vs_oracle or neighbour or c4_plane\[0.0)" > gpurun_out/r05k/tests.log 2>&1 || { tail -30 gpurun_out/r05k/tests.log; exit 1; }
tail -4 gpurun_out/r05k/tests.log
timeout -k 10 400 python -u bench.py --config c4w50 --precision fp64 --steps 5 --warmup 2 --no-cpu-baseline \
  --no-probe --no-reference-precision > gpurun_out/r05k/c4w50_fp64.json 2> gpurun_out/r05k/c4w50_fp64.err || { tail -20 gpurun_out/r05k/c4w50_fp64.err; exit 1; }
python - <<'P'
import json
d=json.loads(open('gpurun_out/r05k/c4w50_fp64.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], {n:(round(v['avg_ms'],2), round((v.get('pmc_bytes_per_launch') or 0)/v['bytes_per_launch'],2)) for n,v in d['kernels'].items()})
P
