#!/usr/bin/env python3
"""Per-kernel-class HBM traffic of the decode kernels from rocprofv3 --pmc CSVs.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch and need separate passes (TCC slots: FETCH_SIZE
takes 3 of 4, WRITE_SIZE 2).  On gfx950 FETCH_SIZE counts exactly half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md, HBM), so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane streaming stores.  Infinity-Cache hits are counted, not excluded.

usage: pmc_traffic.py out.json MODEL:FETCH.csv:WRITE.csv [MODEL:FETCH.csv:WRITE.csv ...]
       MODEL = 7b | 13b; classes of the 13B file are prefixed "13b:" (bench.py looks up
       the 7B dominant kernel's class, e.g. "w13", in this file: --traffic-json).
"""
import csv
import json
import re
import sys
from collections import defaultdict

ALG = {"7b": {"qkv": 31457280, "wo": 10485760, "w13": 56360960, "w2": 28180480, "lm_head": 81920000},
       "13b": {"qkv": 58982400, "wo": 19660800, "w13": 106168320, "w2": 53084160, "lm_head": 122880000}}
EPI_STORE, EPI_RESID, EPI_QKV, EPI_SWIGLU = 0, 1, 2, 4     # lvk_kernels.h epilogue ids


def klass(name):
    m = re.search(r"k_mv_cu<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+)", name)
    if m:                                   # <NW, NP, D, PRO, EPI, KT, PF>
        epi, kt = int(m.group(5)), int(m.group(6))
    else:
        m = re.search(r"k_mv_cu41<(\d+), (\d+), (\d+), (\d+), (\d+)", name)
        if not m:
            if "k_attn_d" in name:
                return "attention"
            return None                     # <NW, D, PRO, EPI, KT, SPLIT>
        epi, kt = int(m.group(4)), int(m.group(5))
    if epi == EPI_QKV:
        return "qkv"
    if epi == EPI_SWIGLU:
        return "w13"
    if epi == EPI_STORE:
        return "lm_head"
    return "wo" if kt in (4096, 5120, 8192) else "w2"


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
    out = {}
    for spec in sys.argv[2:]:
        model, fpath, wpath = spec.split(":")
        fetch = load(fpath, "FETCH_SIZE")
        write = load(wpath, "WRITE_SIZE")
        alg = ALG[model]
        for k, v in fetch.items():
            f = sum(v) / len(v) * 1024 * 2
            w = (sum(write[k]) / len(write[k]) * 1024) if k in write else 0.0
            key = k if model == "7b" else model + ":" + k
            out[key] = {"bytes_per_launch": f + w, "read_bytes": f, "write_bytes": w, "dispatches": len(v),
                        "algorithmic_bytes": alg.get(k),
                        "read_over_algorithmic": (f / alg[k]) if k in alg else None,
                        "method": "rocprofv3 --pmc FETCH_SIZE (KiB x1024 x2, gfx950 half-count correction) and "
                                  "--pmc WRITE_SIZE (KiB x1024) in separate passes, mean per dispatch"}
    json.dump(out, open(sys.argv[1], "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
