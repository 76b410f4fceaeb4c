"""Print the top entries of a cProfile dump (dev tool): python tools/prof_stats.py <file.prof> [n]"""
import pstats
import sys

p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(int(sys.argv[2]) if len(sys.argv) > 2 else 30)
