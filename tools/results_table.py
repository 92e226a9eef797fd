#!/usr/bin/env python3
"""Markdown results table (BASELINE.md / DESIGN.md §5) from committed bench lines and PMC summaries.

    python tools/results_table.py r06_final [r06_v2 r06_v1 ...]

Rows: every profiles/<prefix>_<spec>_bench.json of the first prefix (spec = 2, 2c, 2r10000, ...);
the rocprof average and PMC traffic come from the first of the given prefixes that holds a
profiles/<prefix>_config<C>_pmc.json for the same config and counter setting.
"""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def load(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def spec_key(spec):
    m = re.match(r"(\d+)(?:r(\d+))?(c?)$", spec)
    return (int(m.group(1)), int(m.group(2) or 0), m.group(3)) if m else (99, 0, spec)


def pmc_for(cfg, prefixes):
    for p in prefixes:
        f = os.path.join(PROF, f"{p}_config{cfg}_pmc.json")
        if os.path.exists(f):
            with open(f) as fh:
                return p, json.load(fh)
    return None, None


def main():
    first, rest = sys.argv[1], sys.argv[2:]
    rows = []
    for f in glob.glob(os.path.join(PROF, f"{first}_*_bench.json")):
        spec = os.path.basename(f)[len(first) + 1:-len("_bench.json")]
        if spec.startswith("config"):
            spec = spec[len("config"):]
        if not re.match(r"\d", spec):
            continue
        rows.append((spec_key(spec), spec, load(f)))
    print("| config | workload | rules / tables | tuples | GPU Gpps (bench) | steady | B/tuple | frac of 8 TB/s "
          "(bench / rocprof) | PMC traffic | B2 Mpps (1 / n) | faithful Mpps (1 / n) | parity |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for _, spec, d in sorted(rows):
        c, r, cb = d["config"], d["roofline"], d.get("cpu_baseline") or {}
        cfg = spec.rstrip("c")
        _, pmc = pmc_for(cfg, [first] + rest) if not spec.endswith("c") else (None, None)
        prof = "—"
        traffic = "—"
        if pmc:
            ns = pmc["rocprof_avg_kernel_ns"]
            prof = "%.3f" % (pmc["algorithmic_bytes_per_launch"] / ns / 8000.0)
            traffic = "%.4f" % pmc["traffic_over_algorithmic"]
        st = d.get("steady_state", {}).get("value")
        b2 = "%.2f / %.1f" % (cb["single_thread"]["value"], cb["value"]) if cb.get("single_thread") else "—"
        fa = "%.3g / %.3g" % (cb["faithful_1thread_mpps"], cb["faithful_nthreads_mpps"]) \
            if cb.get("faithful_nthreads_mpps") else "—"
        ps = d.get("parity_sample", {})
        par = "bit-exact" if ps.get("bit_exact_action_and_rule_index") else "MISMATCH"
        if c.get("counters"):
            par += ", counters " + ("equal" if ps.get("counters_equal_oracle_histogram") else "DIFFER")
        print("| %s | %s | %s / %s | %dM | **%.1f**%s | %s | %d | %.3f / %s | %s | %s | %s | %s |" % (
            spec, c["workload"].split(":", 1)[-1].strip()[:48], f"{c['rules']:,}", c["tables"],
            c["tuples_per_gpu"] >> 20, d["value"] / 1000.0, " (counters)" if c.get("counters") else "",
            "%.1f" % (st / 1000.0) if st else "—", r["bytes_per_tuple"], r["frac"], prof, traffic, b2, fa, par))


if __name__ == "__main__":
    main()
