"""Print a kernel timeline (µs, relative) from a rocprofv3 kernel_trace.csv: name filter, window.
python tools/trace_timeline.py <trace.csv> [substring ...] [--skip N] [--count M]"""
import csv
import sys

args = [a for a in sys.argv[2:] if not a.startswith("--")]
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
count = int(sys.argv[sys.argv.index("--count") + 1]) if "--count" in sys.argv else 60
rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if not args or any(a in r["Kernel_Name"] for a in args if not a.isdigit())]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[skip:skip + count]
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:10.1f} {e / 1e3:10.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']} {r['Kernel_Name'][:40]}")
