#!/usr/bin/env python3
"""Summarise tools/pmc_probe.sh passes: per-launch average of every counter for the kernels
whose name matches (default: the classify kernel), plus derived ratios.

    python tools/pmc_table.py gpurun_out/TAG [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_classify"
    for pdir in sorted(glob.glob(os.path.join(d, "pmc_c*_p*"))):
        if not os.path.isdir(pdir):
            continue
        files = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        per = defaultdict(lambda: defaultdict(float))  # (dispatch) -> counter -> sum over dims
        names = {}
        with open(files[0]) as f:
            for r in csv.DictReader(f):
                if pat not in r["Kernel_Name"]:
                    continue
                key = r["Dispatch_Id"]
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
        if not per:
            continue
        keys = sorted(per, key=int)[1:] or sorted(per, key=int)  # drop the first (warm-up) launch
        tot = defaultdict(float)
        for k in keys:
            for c, v in per[k].items():
                tot[c] += v / len(keys)
        print("== %s  (%d launches of %s)" % (os.path.basename(pdir), len(keys), names[keys[0]][:80]))
        for c in sorted(tot):
            print("   %-28s %16.0f" % (c, tot[c]))
        if "SQ_WAVE_CYCLES" in tot:
            w = tot["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in tot:
                    print("   %-28s %15.1f%%" % (c + "/WAVE_CYCLES", 100 * tot[c] / w))


if __name__ == "__main__":
    main()
