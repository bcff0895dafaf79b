set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02n
bash scripts/profile.sh c3 r02n_c3 || exit 1
bash scripts/profile.sh c1 r02n_c1 || exit 1
timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r02n/bench_c1.json 2>gpurun_out/r02n/bench_c1.err || exit 1
timeout -k 10 400 python bench.py --config c2 --steps 10 --warmup 2 > gpurun_out/r02n/bench_c2.json 2>gpurun_out/r02n/bench_c2.err || exit 1
echo all-done
