#!/usr/bin/env python3
"""Per-instantiation register report of the fused kernel (VGPRs, VGPR/SGPR spills).

    python scripts/spills.py [--src FILE] [extra hipcc flags...]

Compiles csrc/dadmm_fused.hip (or csrc/FILE, e.g. --src dadmm_backward.hip; -DDADMM_FUSED_REC=1
for the recording forward) with the Makefile's flags and -Rpass-analysis=kernel-resource-usage
and prints one line per fused_forward_kernel<P, NT, GRAPH, WAVES> instantiation."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd", "csrc", "dadmm_fused.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-slp-vectorize", "-x", "hip", "-c", "-o", "/dev/null",
         "-Rpass-analysis=kernel-resource-usage"]


def main():
    args, src = sys.argv[1:], SRC
    if args[:1] == ["--src"]:
        src, args = os.path.join(os.path.dirname(SRC), args[1]), args[2:]
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *args, src],
                       capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        sys.exit(r.returncode)
    cur, rows = None, {}
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            k = re.search(r"kernelILi(\d+)ELi(\d+)ELi(\d+)E", m.group(1))
            cur = "P=%s NT=%s graph=%s" % k.groups() if k else m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\d+)",
                      line)
        if m and cur:
            rows[cur][m.group(1)] = int(m.group(2))
    for k, v in rows.items():
        print(f"{k:34s} vgpr={v.get('VGPRs', '?'):>4} vspill={v.get('VGPRs Spill', '?'):>4} "
              f"sspill={v.get('SGPRs Spill', '?'):>4} lds={v.get('LDS Size [bytes/block]', '?')}")


if __name__ == "__main__":
    main()
