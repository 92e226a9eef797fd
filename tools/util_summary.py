#!/usr/bin/env python3
"""Utilisation summary of the classify kernel from tools/r02_profile.sh's PMC passes.

Per config (profiles/<prefix>_config<C>_util.json), averaged over the k_classify dispatches
of each pass (counters summed over the chip by rocprofv3):
  clock_ghz        GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration (MI355X_MICROARCH.md DVFS note)
  waves_per_cu     mean resident waves per CU = 4 * SQ_WAVE_CYCLES (quad-cycles) / (CUs * cycles)
  valu_busy        SQ_ACTIVE_INST_VALU * 4 / (SIMDs per CU * CUs * cycles): share of SIMD cycles
                   issuing VALU (the gfx9 VALUBusy formula, which ROCm 7.2 falls back to)
  lds_bank_conflict  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: extra LDS cycles per LDS cycle
  lds_idx_active_per_cu_cycle  SQ_LDS_IDX_ACTIVE / (CUs * cycles) (unit of the counter uncalibrated on gfx950)
  wait_any / wait_inst_any / active_inst_any   shares of SQ_WAVE_CYCLES (disjoint, MICROARCH)
  ta_busy / td_busy   TA_TA_BUSY / TD_TD_BUSY over (CUs * cycles)
  insts per tuple  SQ_INSTS_VALU / _LDS / _VMEM / _SALU per classified tuple (wave instructions x 64 / tuples)
where cycles = GRBM_GUI_ACTIVE / 8 (per XCD) and CUs = 256.

    python tools/util_summary.py gpurun_out/r02_v1 r02_v1
"""
import csv
import glob
import json
import os
import sys

CUS, XCDS, SIMDS = 256, 8, 4


def passes(src, cfg):
    out = {}
    for d in sorted(glob.glob(os.path.join(src, "util_c%s_p*" % cfg))):
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        per, names = {}, {}
        rows = [r for r in csv.DictReader(open(f[0])) if "k_classify" in r["Kernel_Name"]]
        for r in rows:
            names.setdefault(r["Kernel_Name"], set()).add(r["Dispatch_Id"])
        # the config's own kernel: the k_classify dispatched most often (the default config-2
        # line also times its side blocks' kernels, fewer times each)
        kname = max(names, key=lambda k: len(names[k])) if names else None
        for r in rows:
            if r["Kernel_Name"] != kname:
                continue
            key = int(r["Dispatch_Id"])
            e = per.setdefault(key, {"dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if per:
            out[os.path.basename(d)] = list(per.values())
    return out


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for bench in sorted(glob.glob(os.path.join(src, "bench_c*.json"))):
        cfg = os.path.basename(bench)[len("bench_c"):-len(".json")]
        line = json.loads(open(bench).read().strip().splitlines()[-1])
        n = line["config"]["tuples_per_gpu"]
        res = {"config": int(cfg) if cfg.isdigit() else cfg, "tuples_per_launch": n, "passes": {}}
        acc = {}
        for name, ds in passes(src, cfg).items():
            avg = {k: sum(d.get(k, 0.0) for d in ds) / len(ds) for k in ds[0]}
            res["passes"][name] = {k: round(v, 1) for k, v in avg.items()}
            for k, v in avg.items():
                acc.setdefault(k, v)
        if not acc:
            continue
        cyc = acc["GRBM_GUI_ACTIVE"] / XCDS
        g = lambda k: acc.get(k)  # noqa: E731
        m = {"clock_ghz": round(acc["GRBM_GUI_ACTIVE"] / XCDS / acc["dur"], 3)}
        if g("SQ_WAVE_CYCLES"):
            m["waves_per_cu"] = round(4 * g("SQ_WAVE_CYCLES") / (CUS * cyc), 2)
        if g("SQ_ACTIVE_INST_VALU"):
            m["valu_busy"] = round(4 * g("SQ_ACTIVE_INST_VALU") / (SIMDS * CUS * cyc), 4)
        if g("SQ_LDS_IDX_ACTIVE"):
            m["lds_idx_active_per_cu_cycle"] = round(g("SQ_LDS_IDX_ACTIVE") / (CUS * cyc), 4)
            m["lds_bank_conflict"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 4)
        if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                m[k.lower()[3:]] = round(g(k) / g("SQ_WAVE_CYCLES"), 4)
        for k in ("TA_TA_BUSY", "TD_TD_BUSY"):
            if g(k):
                m[k.lower()[3:]] = round(g(k) / (CUS * cyc), 4)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU"):
            if g(k):
                m["wave_insts_per_64_tuples_" + k[9:].lower()] = round(g(k) * 64 / n, 2)
        res["metrics"] = m
        res["note"] = __doc__.split("\n\n")[1]
        out = os.path.join(root, "profiles", "%s_config%s_util.json" % (prefix, cfg))
        json.dump(res, open(out, "w"), indent=1)
        print(cfg, json.dumps(m))


if __name__ == "__main__":
    main()
