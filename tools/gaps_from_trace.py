"""Mean gap (next start - previous end) per consecutive kernel pair in a rocprofv3 kernel trace CSV."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
gaps, durs = collections.defaultdict(list), collections.defaultdict(list)
short = lambda n: n.split("(")[0].replace("void ", "")[:40]
for a, b in zip(rows[skip:], rows[skip + 1:]):
    gaps[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in rows[skip:]:
    durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(durs.items()):
    print(f"dur  {k:42s} {sum(v)/len(v):9.2f} us  n={len(v)}")
for k, v in sorted(gaps.items()):
    print(f"gap  {k[0]:30s} -> {k[1]:30s} {sum(v)/len(v):8.2f} us  n={len(v)}")
