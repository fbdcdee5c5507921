#!/usr/bin/env python3
"""Copy engines vs blit kernels in a rocprofv3 --kernel-trace --memory-copy-trace database: per copy
direction the count, bytes and summed time of the memory-copy records, and the blit kernels
(__amd_rocclr_copy*) of the same run."""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")]
    print("tables/views:", ", ".join(sorted(n for n in names if not n.startswith("sqlite"))))
    for view in ("memory_copies", "memory_copy"):
        if view in names:
            cols = [r[1] for r in c.execute("pragma table_info(%s)" % view)]
            print(view, "columns:", cols)
            key = next((k for k in ("name", "kind", "direction", "src_agent_type") if k in cols), None)
            size = next((k for k in ("size", "bytes") if k in cols), None)
            q = "select %s, count(*), %s, sum(duration) from %s group by %s" % (
                key or "'all'", "sum(%s)" % size if size else "0", view, key or "'all'")
            for row in c.execute(q):
                print("  copy", row)
            break
    for n, k, t in c.execute("select name, count(*), sum(duration) from kernels where name like '%rocclr%' group by name"):
        print("  blit kernel %s: %d calls, %.3f ms" % (n, k, t / 1e6))


if __name__ == "__main__":
    main(sys.argv[1])
