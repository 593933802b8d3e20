"""Per-kernel average durations from rocprofv3 databases (tools/prof_kt.sh output).
usage: python tools/kt_summary.py gpurun_out/TAG_cur gpurun_out/TAG_var ... [-k SUBSTR]"""
import argparse
import glob
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("-k", default="", help="kernel-name substring filter")
ap.add_argument("--top", type=int, default=12)
a = ap.parse_args()
for d in a.dirs:
    db = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(end-start), sum(end-start) from kernels "
                     "group by name order by sum(end-start) desc").fetchall()
    print(f"== {d}")
    for name, cnt, avg, tot in [r for r in rows if a.k in r[0]][: a.top]:
        print(f"  {name[:72]:72s} {cnt:5d} {avg / 1e3:10.1f} us")
