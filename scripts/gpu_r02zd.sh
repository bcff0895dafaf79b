set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02zd
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02zd/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-pmc --no-cpu-baseline --no-probe > gpurun_out/r02zd/bench.json 2>/dev/null || exit 1
echo all-done
