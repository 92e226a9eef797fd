#!/usr/bin/env python3
"""Turn a tools/gpu_check.sh output directory into the committed profile summaries.

For every config C found in gpurun_out/TAG/:
  profiles/<prefix>_config<C>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<prefix>_config<C>_pmc.json           FETCH_SIZE / WRITE_SIZE per classify launch
  profiles/<prefix>_config<C>_bench.json         the bench line of the same box

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE come from separate passes (they cannot share the 4 TCC slots),
are reported in KiB, and on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
streaming reads, so the stream part is doubled. The classify kernel's tuple streams are
16/8/4-byte-per-lane loads; any table-blob reads that miss L2 (config 4) are not wide
streams, so `fetch_stream_bytes_corrected` is reported next to the raw figure.

    python tools/prof_summary.py gpurun_out/v3 r01_v3
"""
import csv
import glob
import json
import os
import shutil
import sqlite3
import sys


def _db(path):
    f = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    return sqlite3.connect(f[0]) if f else None


def kernel_stats(prof_dir, out_csv):
    stats = glob.glob(os.path.join(prof_dir, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], out_csv)
        with open(stats[0]) as f:
            return list(csv.DictReader(f))
    c = _db(prof_dir)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"]
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(hdr)
        for r in rows:
            # top_kernels durations are in microseconds
            w.writerow([r[0], r[1], round(r[2] * 1e3), round(r[3] * 1e3, 1), round(r[4], 3)])
    return [dict(zip(hdr, [r[0], r[1], r[2] * 1e3, r[3] * 1e3, r[4]])) for r in rows]


def pmc_values(pmc_dir, counter):
    c = _db(pmc_dir)
    if c is not None:
        rows = c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                         (counter,)).fetchall()
    else:
        f = glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)[0]
        with open(f) as fh:
            rows = [(r["Kernel_Name"], float(r["Counter_Value"])) for r in csv.DictReader(fh)
                    if r["Counter_Name"] == counter]
    out = {}
    for name, v in rows:
        out.setdefault(name, []).append(float(v))
    return out


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    for bench in sorted(glob.glob(os.path.join(src, "bench_c*.json"))):
        cfg = os.path.basename(bench)[len("bench_c"):-len(".json")]
        shutil.copy(bench, os.path.join(prof, f"{prefix}_config{cfg}_bench.json"))
        with open(bench) as f:
            line = json.loads(f.read().strip().splitlines()[-1])
        stats = kernel_stats(os.path.join(src, f"prof_c{cfg}"),
                             os.path.join(prof, f"{prefix}_config{cfg}_kernel_stats.csv"))
        fetch = pmc_values(os.path.join(src, f"pmc_FETCH_SIZE_c{cfg}"), "FETCH_SIZE")
        write = pmc_values(os.path.join(src, f"pmc_WRITE_SIZE_c{cfg}"), "WRITE_SIZE")
        # the config's own kernel: the k_classify launched most often (the default config-2 line
        # also times its side blocks' kernels, fewer times each)
        kname = max((k for k in fetch if "k_classify" in k), key=lambda k: len(fetch[k]))
        avg = lambda xs: sum(xs) / len(xs)
        f_raw = avg(fetch[kname]) * 1024
        w_raw = avg(write[kname]) * 1024
        n = line["config"]["tuples_per_gpu"]
        stream_read = n * (line["roofline"]["bytes_per_tuple"] - 4)
        algo = n * line["roofline"]["bytes_per_tuple"]
        prof_avg_ns = next(float(s["AverageNs"]) for s in stats if s["Name"] == kname)
        # the tuple streams show up at half their bytes; whatever FETCH_SIZE holds beyond
        # that is table-blob (L2-miss) reads, taken at face value (uncalibrated width)
        stream_raw = min(f_raw, stream_read / 2)
        other_raw = f_raw - stream_raw
        traffic = 2 * stream_raw + other_raw + w_raw
        summary = {
            "config": int(cfg) if cfg.isdigit() else cfg, "kernel": kname, "launches_sampled": len(fetch[kname]),
            "tuples_per_launch": n, "algorithmic_bytes_per_launch": algo,
            "fetch_size_raw_bytes": round(f_raw), "write_size_bytes": round(w_raw),
            "fetch_stream_bytes_corrected": round(2 * stream_raw),
            "fetch_table_bytes_raw": round(other_raw),
            "hbm_traffic_bytes_per_launch": round(traffic),
            "traffic_over_algorithmic": round(traffic / algo, 4),
            "algorithmic_stream_read_bytes": stream_read,
            "rocprof_avg_kernel_ns": prof_avg_ns,
            "bench_kernel_ms": line["roofline"]["kernel_ms"],
            "note": ("tuple-stream part of FETCH_SIZE doubled per the gfx950 correction for wide "
                     "streaming reads; the remainder (table blob reads missing L2, served by the "
                     "Infinity Cache or HBM) taken as reported"),
        }
        with open(os.path.join(prof, f"{prefix}_config{cfg}_pmc.json"), "w") as f:
            json.dump(summary, f, indent=1)
        print(json.dumps(summary))


if __name__ == "__main__":
    main()
