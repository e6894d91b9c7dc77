#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc counter_collection.csv files per kernel name: dispatch count and
the mean value per dispatch of every counter.  usage: pmc_reduce.py out.json a.csv [b.csv ...]
(FETCH_SIZE is additionally reported doubled as fetch_bytes, the gfx950 half-count correction
of MI355X_MICROARCH.md; WRITE_SIZE as write_bytes, both KiB -> bytes)."""
import csv
import json
import sys
from collections import defaultdict


def main():
    out = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[2:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].replace("(anonymous namespace)", "(anon)")
            name = name.split("(lvk::")[0].split("(unsigned")[0].split("(float")[0].split("(const")[0]
            out[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for name, cs in out.items():
        d = {"dispatches": max(len(v) for v in cs.values())}
        for c, v in cs.items():
            d[c] = sum(v) / len(v)
        if "FETCH_SIZE" in d:
            d["fetch_bytes"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024
        res[name] = d
    json.dump(res, open(sys.argv[1], "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
