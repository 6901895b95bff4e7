#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (--kernel-trace --stats) into a per-kernel CSV:
name, calls, total/avg/min/max duration (us), VGPR/AGPR/SGPR, LDS, scratch, grid."""
import csv
import glob
import sqlite3
import sys


def main(db_glob: str, out_csv: str):
    db = sorted(glob.glob(db_glob, recursive=True))[0]
    con = sqlite3.connect(db)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size), "
        "max(grid_x), max(workgroup_x) from kernels group by name order by sum(duration) desc").fetchall()
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "vgpr", "agpr", "sgpr", "lds_bytes",
                    "scratch_bytes", "grid_x", "workgroup_x"])
        for r in rows:
            name = r[0].split("(")[0]
            w.writerow([name, r[1]] + [round(x / 1e3, 3) for x in r[2:6]] + list(r[6:]))
    print(open(out_csv).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
