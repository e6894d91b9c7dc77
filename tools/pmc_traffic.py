#!/usr/bin/env python3
"""Per-kernel-class HBM traffic from rocprofv3 --pmc CSVs (FETCH_SIZE, WRITE_SIZE passes).

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts exactly half
the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM), so it is doubled.
Usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv > profiles/rNN_traffic.json
"""
import csv
import json
import re
import sys
from collections import defaultdict

ALG = {"qkv": 31457280, "wo": 10485760, "w13": 56360960, "w2": 28180480, "lm_head": 81920000}


def klass(name):
    m = re.search(r"k_mv_cu<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", name)
    if m:
        pro, epi, kt = int(m.group(4)), int(m.group(5)), int(m.group(6))
        return {2: "qkv", 4: "w13", 0: "lm_head"}.get(epi) or ("wo" if kt == 4096 else "w2")
    if "k_attn_wo" in name:
        return "attn_wo"
    if "k_attn" in name:
        return "attention"
    return None


def load(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = klass(r["Kernel_Name"])
        if k:
            acc[k].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE") if len(sys.argv) > 2 else {}
    out = {}
    for k, v in fetch.items():
        f = sum(v) / len(v) * 1024 * 2
        w = (sum(write[k]) / len(write[k]) * 1024) if k in write else 0.0
        out[k] = {"bytes_per_launch": f + w, "read_bytes": f, "write_bytes": w, "dispatches": len(v),
                  "algorithmic_bytes": ALG.get(k), "read_over_algorithmic": (f / ALG[k]) if k in ALG else None,
                  "method": "rocprofv3 --pmc FETCH_SIZE (x1024 x2, gfx950 half-count correction) + WRITE_SIZE (x1024)"}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
