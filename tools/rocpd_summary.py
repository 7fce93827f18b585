"""Per-kernel summary of a rocprofv3 sqlite output (kernel trace and --pmc passes): mean
duration and dispatches per kernel, and each counter summed per dispatch (measurement tool).

  python tools/rocpd_summary.py DB [DB ...] [--kernel REGEX]
"""
import argparse
import re
import sqlite3


def short(name):
    """a kernel's name without the namespace noise and the parameter list"""
    n = name.replace("(anonymous namespace)::", "")
    return n.split("(")[0][-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--kernel", default=".")
    a = ap.parse_args()
    kre = re.compile(a.kernel)
    for db in a.dbs:
        c = sqlite3.connect(db)
        print("==", db)
        for name, n, avg in c.execute("select name, count(*), avg(end-start) from kernels group by name order by 3 desc"):
            if kre.search(name):
                print("  %-60s n=%-4d mean %.4f ms" % (short(name), n, avg / 1e6))
        rows = c.execute("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) from counters_collection "
                         "group by kernel_name, counter_name").fetchall()
        for k, cn, v, nd in rows:
            if kre.search(k):
                print("  %-40s %-24s %.4g per dispatch" % (short(k)[-40:], cn, v / nd))


if __name__ == "__main__":
    main()
