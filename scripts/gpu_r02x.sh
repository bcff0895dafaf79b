set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02x
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$GRAFT_REPO_ROOT/bench.py --config c3 --steps 4 --warmup 0 --no-cpu-baseline --no-pmc --no-probe"
PDHG_FUSE_RES=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/nofuse -o run -- python3 $ARGS > $OUT/nofuse.log 2>&1 || exit 1
echo all-done
