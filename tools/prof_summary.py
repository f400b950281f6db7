#!/usr/bin/env python3
"""Summarise a tools/profile.sh output dir: per (kernel, grid) average duration from the kernel
trace, FETCH_SIZE / WRITE_SIZE per launch from the PMC passes (gfx950: FETCH_SIZE reads 1/2 of a
wide coalesced stream's bytes -> reported x2 as 'hbm_read_MB_corr')."""
import collections
import csv
import sys

d = sys.argv[1]


def key(r, grid):
    return (r["Kernel_Name"].split("(")[0][:58], grid)


tr = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")):
    g = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    tr[key(r, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))


def pmc(sub):
    out = collections.defaultdict(list)
    try:
        for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
            out[key(r, r["Grid_Size"])].append(float(r["Counter_Value"]))
    except FileNotFoundError:
        pass
    return out


fe, wr = pmc("fetch"), pmc("write")
# pmc grid is total threads; map by kernel name + order-insensitive mean
fe_n = collections.defaultdict(list)
wr_n = collections.defaultdict(list)
for (n, g), v in fe.items():
    fe_n[n] += v
for (n, g), v in wr.items():
    wr_n[n] += v
tot = sum(sum(v) for v in tr.values())
print(f"{'kernel':58s} {'grid':>14s} {'n':>4s} {'avg_us':>9s} {'share':>6s}")
for k in sorted(tr, key=lambda k: -sum(tr[k]))[:18]:
    v = tr[k]
    print(f"{k[0]:58s} {k[1]:>14s} {len(v):4d} {sum(v)/len(v)/1e3:9.1f} {100*sum(v)/tot:5.1f}%")
print()
print(f"{'kernel':58s} {'FETCH_MB':>10s} {'x2corr':>10s} {'WRITE_MB':>10s}  (mean per launch over all grids)")
for n in sorted(fe_n, key=lambda n: -sum(fe_n[n]))[:12]:
    f = sum(fe_n[n]) / len(fe_n[n]) / 1024
    w = sum(wr_n[n]) / len(wr_n[n]) / 1024 if wr_n.get(n) else 0.0
    print(f"{n:58s} {f:10.1f} {2*f:10.1f} {w:10.1f}")
