"""Host-side profile of the marching time-to-solution run (GPU box): cProfile around bench.py --marching, the top
entries by own time.  usage: python scripts/prof_host_marching.py [bench args]"""
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import bench  # noqa: E402

sys.argv = ["bench.py", "--config", "c2", "--marching", "--rho-alp-iters", "10", "--no-cpu-baseline"] + sys.argv[1:]
pr = cProfile.Profile()
pr.enable()
try:
    bench.main()
finally:
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)
