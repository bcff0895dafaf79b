# round 2 profiles: rocprofv3 kernel trace + PMC for C3 and C1, full default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02g
timeout -k 10 900 bash scripts/profile.sh c3 r02_c3 > gpurun_out/r02g/prof_c3.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/profile.sh c1 r02_c1 > gpurun_out/r02g/prof_c1.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/r02g/bench_c3_full.json 2> gpurun_out/r02g/bench_c3_full.err || exit 1
echo all-done
