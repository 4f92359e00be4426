#!/usr/bin/env python3
"""Timed-region structure of a bench kernel trace: pixel launch periods, the last batch's tail,
and every kernel from a window before the last pixel launch.  Usage: tools/timeline_tail.py trace.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pix = [r for r in rows if "k_pix5" in r["Kernel_Name"] or "k_pixw" in r["Kernel_Name"]]
tp = pix[-steps:]
s0 = int(tp[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in rows if "fm::" in r["Kernel_Name"])
per = [(int(tp[i + 1]["Start_Timestamp"]) - int(tp[i]["Start_Timestamp"])) / 1e3 for i in range(len(tp) - 1)]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tp]
print(f"timed span {(end - s0) / 1e3:.1f} us for {steps} batches = {(end - s0) / 1e3 / steps:.1f} us/step")
print("pixel periods", [round(p) for p in per])
print("pixel durations", [round(d) for d in dur])
le = int(tp[-1]["End_Timestamp"])
print(f"tail after the last pixel launch {(end - le) / 1e3:.1f} us")
ls = int(tp[-1]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e > ls - 100000 and "fm::" in r["Kernel_Name"]:
        print(f"{(s - ls) / 1e3:8.1f} {(e - ls) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:34]}")
