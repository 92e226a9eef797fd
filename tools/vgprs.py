#!/usr/bin/env python3
"""Per-kernel VGPR / occupancy report of device.hip (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/vgprs.py [-DMACRO=...]   -> "kernel-template-args VGPRs occupancy" lines
"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-parameter",
       "-Rpass-analysis=kernel-resource-usage", "-c", "vpp_amd/csrc/device.hip", "-o", "/tmp/vgprs_probe.o"] + sys.argv[1:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    m = re.search(r"k_classifyILi(\d)ELb(\d)ELb(\d)ELi(\d+)ELb(\d)ELi(\d+)E", k)
    name = "classify<M%s C%s V%s S%s N%s %s>" % m.groups() if m else k[:40]
    print("%-32s vgpr %3d occ %2d scratch %d" % (name, v.get("VGPRs", -1), v.get("Occupancy [waves/SIMD]", -1),
                                                   v.get("ScratchSize [bytes/lane]", -1)))
