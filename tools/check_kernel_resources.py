#!/usr/bin/env python3
"""Build gate: parse hipcc's -Rpass-analysis=kernel-resource-usage remarks and fail when an SDDMM
kernel (k_sddmm*, k_sim_filter) spills VGPRs/SGPRs or uses scratch. Usage: check_kernel_resources.py <remarks>"""
import os
import re
import sys


def main(path):
    kern, bad, seen = None, [], 0
    with open(path, errors="replace") as f:
        for line in f:
            m = re.search(r"remark:\s+Function Name: (\S+)", line)
            if m:
                kern = m.group(1)
                seen += "k_sddmm" in kern or "k_sim_filter" in kern
                continue
            if not kern or ("k_sddmm" not in kern and "k_sim_filter" not in kern):
                continue
            allow = os.environ.get("RES_CHECK_ALLOW")  # experiments only: a regex of kernels
            if allow and re.search(allow, kern):
                continue
            m = re.search(r"remark:\s+(VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]): (\d+)",
                          line)
            if m and int(m.group(2)) > 0:
                bad.append(f"{kern}: {m.group(1)} = {m.group(2)}")
    if bad:
        sys.stderr.write("kernel resource check failed (spills/scratch):\n  " + "\n  ".join(bad) + "\n")
        return 1
    if seen == 0:
        sys.stderr.write(f"kernel resource check: no k_sddmm / k_sim_filter kernels in {path}\n")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
