"""Dev tool: per-token timeline of a decode run from rocprofv3 traces.

usage: timeline.py <dir with *kernel_trace.csv [*memory_copy_trace.csv]> [first_kernel_substring]

Splits the kernel trace into tokens at every launch of the first kernel of a token (default
the embedding kernel), then reports per token: span (first start -> last end), the sum of
kernel durations, the idle time between kernels inside the token, the idle time from the end
of one token to the start of the next, and the largest inner gaps with the kernels around
them.  Memory copies (when traced) are listed with their durations."""
import csv
import glob
import os
import statistics
import sys


def load(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    d = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_embed"
    ks = load(os.path.join(d, "**", "*kernel_trace.csv"))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ks]
    ks.sort()
    cps = load(os.path.join(d, "**", "*memory_copy_trace.csv"))
    cps = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Kind", "")))
                 for r in cps)
    toks, cur = [], []
    for k in ks:
        if first in k[2] and cur:
            toks.append(cur)
            cur = []
        cur.append(k)
    if cur:
        toks.append(cur)
    toks = [t for t in toks if first in t[0][2]]
    if len(toks) < 3:
        print("fewer than 3 tokens found")
        return
    toks = toks[1:-1]       # drop partial first/last
    spans, busy, inner, between, gaps = [], [], [], [], {}
    for i, t in enumerate(toks):
        spans.append(t[-1][1] - t[0][0])
        busy.append(sum(e - s for s, e, _ in t))
        g = 0
        for a, b in zip(t, t[1:]):
            dg = max(0, b[0] - a[1])
            g += dg
            key = (short(a[2]), short(b[2]))
            gaps.setdefault(key, []).append(dg)
        inner.append(g)
        if i + 1 < len(toks):
            between.append(toks[i + 1][0][0] - t[-1][1])
    us = lambda v: statistics.median(v) / 1e3
    print("tokens %d  kernels/token %d" % (len(toks), len(toks[0])))
    print("median per token (us): span %.1f  kernel busy %.1f  inner gaps %.1f  end->next start %.1f  period %.1f" %
          (us(spans), us(busy), us(inner), us(between) if between else 0, us(spans) + (us(between) if between else 0)))
    print("inner gap by kernel pair (median us x count per token):")
    n = len(toks)
    for key, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print("  %-28s -> %-28s %6.2f x %d" % (key[0], key[1], statistics.median(v) / 1e3, len(v) // n))
    if cps:
        print("memory copies (median us): %s" % ", ".join(
            "%s %.1f" % (k, statistics.median([e - s for s, e, kk in cps if kk == k]) / 1e3) for k in sorted({c[2] for c in cps})))
        # position of copies relative to the kernels of a token
        t = toks[len(toks) // 2]
        near = [c for c in cps if t[0][0] - 200000 <= c[0] <= t[-1][1] + 200000]
        for s, e, k in near:
            print("  copy %s start %+.1f us from token start, %.1f us" % (k, (s - t[0][0]) / 1e3, (e - s) / 1e3))


def short(name):
    name = name.split("(")[0]
    for p in ("void ", "lvk::", "(anonymous namespace)::"):
        name = name.replace(p, "")
    return name[:28]


if __name__ == "__main__":
    main()
