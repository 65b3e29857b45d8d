"""Print the top functions (tottime) of cProfile dumps side by side.
Usage: python tools/prof_cmp.py A.prof [B.prof ...]"""
import pstats
import sys

for f in sys.argv[1:]:
    print("==", f)
    st = pstats.Stats(f)
    st.sort_stats("tottime").print_stats(18)
