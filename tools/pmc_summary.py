#!/usr/bin/env python3
"""Summarise rocprofv3 PMC pass directories (CSV) per kernel: mean counter
value per dispatch, plus derived ratios.  usage: pmc_summary.py DIR [kernel-substr...]"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"orx::(\w+(<\w+>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:30]
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(per.items()):
        if want and not any(w in k for w in want):
            continue
        v = {c: sum(x) / len(x) for c, x in cs.items()}
        print(f"== {k}")
        for c in sorted(v):
            print(f"   {c:28s} {v[c]:16.1f}")
        if "SQ_WAVE_CYCLES" in v and "SQ_WAIT_ANY" in v:
            wc = v["SQ_WAVE_CYCLES"]
            print(f"   wait_any/wave_cycles {v['SQ_WAIT_ANY'] / wc:.3f}  active/wave_cycles "
                  f"{v.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}")
        if "TCC_HIT_sum" in v:
            print(f"   L2 hit rate {v['TCC_HIT_sum'] / max(1, v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.3f}")
        if "SQ_INSTS_VALU" in v and "SQ_WAVES" in v:
            print(f"   VALU/wave {v['SQ_INSTS_VALU'] / v['SQ_WAVES']:.0f}  VMEM_RD/wave {v.get('SQ_INSTS_VMEM_RD', 0) / v['SQ_WAVES']:.0f}")


if __name__ == "__main__":
    main()
