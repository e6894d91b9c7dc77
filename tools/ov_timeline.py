"""Dev tool (round 6): per-layer edge timing of the decode from a rocprofv3 kernel trace:
for every attention launch, its duration, the following Wo's start / end relative to the
attention's end, and the gap to the next launch.  usage: ov_timeline.py <trace dir>"""
import csv
import glob
import os
import statistics
import sys


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    out = {"att": [], "wo_start_rel": [], "wo_end_rel": [], "wo_dur": [], "w13_start_rel_wo_end": [],
           "qkv_end_to_att_start": []}
    for i, (s, e, n) in enumerate(ks):
        if "k_attn_d" in n and i + 2 < len(ks) and "k_mv_cu" in ks[i + 1][2]:
            out["att"].append((e - s) / 1e3)
            ws, we, _ = ks[i + 1]
            out["wo_start_rel"].append((ws - e) / 1e3)
            out["wo_end_rel"].append((we - e) / 1e3)
            out["wo_dur"].append((we - ws) / 1e3)
            out["w13_start_rel_wo_end"].append((ks[i + 2][0] - we) / 1e3)
            out["qkv_end_to_att_start"].append((s - ks[i - 1][1]) / 1e3)
    for k, v in out.items():
        if v:
            print("%-22s n %4d median %7.2f us  p10 %7.2f  p90 %7.2f" % (k, len(v), statistics.median(v),
                  sorted(v)[len(v) // 10], sorted(v)[9 * len(v) // 10]))


if __name__ == "__main__":
    main()
