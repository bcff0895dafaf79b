#!/bin/bash
# round 5: marching time-to-solution record (C2 fp64, first 10 windows) + a rocprofv3 summary of 2 windows
set -o pipefail
mkdir -p gpurun_out/r05s
timeout -k 10 300 python -u bench.py --config c2 --marching --rho-alp-iters 10 --windows 10 --no-cpu-baseline \
  > gpurun_out/r05s/march10.json 2> gpurun_out/r05s/march10.err || { tail -5 gpurun_out/r05s/march10.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r05s/march10.json').read().strip().splitlines()[-1]); print(d['value'], d['total_outer_iters'], d['ms_per_outer_iter'], d['iters_per_window_first10'])"
bash scripts/prof_marching.sh r05 --windows 2 && python scripts/rocpd_stats.py gpurun_out/prof_r05/trace/run_results.db gpurun_out/r05s/march2_stats.csv 2>/dev/null; ls gpurun_out/prof_r05/trace
