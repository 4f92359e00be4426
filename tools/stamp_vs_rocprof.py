#!/usr/bin/env python3
"""stamp_vs_rocprof.py PROFDIR [KERNEL_SUBSTR] -- the bench line's in-kernel launch stamps against rocprofv3's
kernel trace of the SAME run (tools/profile.sh: PROFDIR/trace.log holds the line, PROFDIR/trace/ the trace):
the average over the timed launches (the last `launches_timed` of the kernel) from both clocks."""
import csv
import glob
import json
import sys


def main(d, kern=None):
    line = [l for l in open(f"{d}/trace.log") if l.startswith("{")][-1]
    js = json.loads(line)
    roof = js["roofline"]
    kern = kern or {"pix": "k_pix5", "resize_area": "k_resize_area"}.get(roof["kernel"], roof["kernel"])
    n = roof["launches_timed"]
    rows = []
    for f in glob.glob(f"{d}/trace/*kernel_trace.csv"):
        rows += [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
    tail = dur[-n:]
    rp = sum(tail) / len(tail)
    print(f"kernel {kern}: bench stamps {roof['avg_launch_us']:.1f} us over {n} timed launches; rocprofv3 "
          f"{rp:.1f} us over the same last {len(tail)} launches ({len(dur)} in the run, all-launch mean "
          f"{sum(dur) / len(dur):.1f}); stamps / rocprof = {roof['avg_launch_us'] / rp:.4f}; "
          f"frac {roof['frac']} (stamps) vs {roof['frac'] * roof['avg_launch_us'] / rp:.4f} (rocprof)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
