#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 results database (average duration in ms)."""
import glob
import sqlite3
import sys

for db in glob.glob(sys.argv[1] + "/**/*.db", recursive=True):
    c = sqlite3.connect(db)
    for name, calls, avg in c.execute("select name, total_calls, average from top_kernels limit %d" % (int(sys.argv[2]) if len(sys.argv) > 2 else 6)):
        print(f"{name[:48]:48s} {calls:5d} {avg / 1e3:9.3f} ms")
