#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS / occupancy table of the engine for gfx950.

Compiles csrc/bcsim_capi.hip (device only) with -Rpass-analysis=kernel-resource-usage and
prints one Markdown row per kernel instantiation (demangled with c++filt), scratch first.
  python3 tools/resource_usage.py > profiles/rNN_resource_usage.md
"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "blockchain-simulator_amd")
FIELDS = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
          "VGPRs Spill", "SGPRs Spill", "LDS Size [bytes/block]")


def main():
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    with tempfile.TemporaryDirectory() as td:
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I../include", "-c",
               "csrc/bcsim_capi.hip", "-o", os.path.join(td, "x.o"), "--offload-device-only",
               "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-4000:])
        return 1
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z][^:]*): (\S+) \[-Rpass", line)
        if m and cur is not None and m.group(1) in FIELDS:
            cur[m.group(1)] = m.group(2)
    names = [x["name"] for x in rows]
    try:  # (binutils c++filt; the ROCm LLVM tree ships no llvm-cxxfilt)
        dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    except OSError:
        dem = names
    for x, d in zip(rows, dem):
        x["name"] = re.sub(r"\(.*\)$", "", d).replace("bcsim::", "").replace("void ", "")
    rows.sort(key=lambda x: (-int(x.get("ScratchSize [bytes/lane]", 0)), x["name"]))
    print("| kernel | VGPRs | AGPRs | SGPRs | scratch B/lane | waves/SIMD | LDS B/block |")
    print("|---|---|---|---|---|---|---|")
    for x in rows:
        print(f"| `{x['name']}` | {x.get('VGPRs')} | {x.get('AGPRs')} | {x.get('TotalSGPRs')} | "
              f"{x.get('ScratchSize [bytes/lane]')} | {x.get('Occupancy [waves/SIMD]')} | {x.get('LDS Size [bytes/block]')} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
