set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02m
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r02m/suite.log 2>&1; echo "suite rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02m/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/r02m/bench_default.json 2>gpurun_out/r02m/bench_default.err || exit 1
timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 > gpurun_out/r02m/bench_c1.json 2>gpurun_out/r02m/bench_c1.err || exit 1
echo all-done
