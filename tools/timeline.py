#!/usr/bin/env python3
"""Print the tail of a rocprofv3 kernel trace as a timeline (us) and the pixel-kernel gaps."""
import csv, glob, os, sys
d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
pix = [r for r in rows if "k_pix" in r["Kernel_Name"]]
for r in rows[-70:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s/1e3:10.1f} {e/1e3:10.1f} {(e-s)/1e3:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:48]}")
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(pix[-16:], pix[-15:])]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in pix[-16:]]
print("pix durations", [round(x, 1) for x in durs])
print("pix gaps", [round(x, 1) for x in gaps])
