#!/usr/bin/env python3
"""Per-kernel SQ counter summary of tools/pmc_bench.sh output (normalised per launch)."""
import collections
import csv
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
dur = collections.defaultdict(dict)
for sub in ("a", "b"):
    try:
        rows = list(csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")))
    except FileNotFoundError:
        continue
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:50]
        agg[n][r["Counter_Name"] + "@" + sub] += float(r["Counter_Value"])
        cnt[n].add((sub, r["Dispatch_Id"]))
        dur[n][(sub, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for n in sorted(agg, key=lambda n: -sum(dur[n].values()))[:8]:
    a = agg[n]
    na = len([1 for s, _ in cnt[n] if s == "a"]) or 1
    nb = len([1 for s, _ in cnt[n] if s == "b"]) or 1
    da = sum(v for (s, _), v in dur[n].items() if s == "a") / na
    g = lambda k, s="a": a.get(k + "@" + s, 0.0) / (na if s == "a" else nb)
    clk = g("GRBM_GUI_ACTIVE") / 8 / da if da else 0
    cyc = da * clk  # kernel cycles at the effective clock
    print(f"{n}: dur {da/1e3:.1f} us, clk {clk:.2f} GHz")
    print(f"   MFMA busy / (1024 SIMD x cycles): {g('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * cyc):.2f}")
    print(f"   insts per launch: VALU {g('SQ_INSTS_VALU'):.3g}  MFMA {g('SQ_INSTS_MFMA'):.3g}  LDS {g('SQ_INSTS_LDS'):.3g}")
    wc = g("SQ_WAVE_CYCLES")
    print(f"   ACTIVE_INST_VALU/WAVE_CYCLES {g('SQ_ACTIVE_INST_VALU')/wc:.2f}")
    wcb = g("SQ_WAIT_ANY", "b") + g("SQ_WAIT_INST_ANY", "b") + g("SQ_ACTIVE_INST_ANY", "b")
    if wcb:
        print(f"   wait_any {g('SQ_WAIT_ANY','b')/wcb:.2f} wait_inst {g('SQ_WAIT_INST_ANY','b')/wcb:.2f} (lds {g('SQ_WAIT_INST_LDS','b')/wcb:.2f}) active {g('SQ_ACTIVE_INST_ANY','b')/wcb:.2f}"
              f"  lds_bank_conflict/active_lds {g('SQ_LDS_BANK_CONFLICT','b')/max(g('SQ_ACTIVE_INST_LDS','b'),1):.2f}  vmem_cyc {g('SQ_INST_CYCLES_VMEM','b'):.3g}")
