#!/usr/bin/env python3
"""HBM traffic per SDDMM launch from a tools/gpu_pmc.sh run (separate FETCH_SIZE and WRITE_SIZE
passes over tools/prof_sddmm.py), corrected as MI355X_MICROARCH.md's HBM section prescribes:
FETCH_SIZE (KiB) reports half the bytes of wide reads on gfx950 -> x2; WRITE_SIZE (KiB) as is
(exact for 16-B streaming stores; the 4-byte scattered output stores are an uncalibrated width).
Writes the JSON bench.py reads for roofline.traffic.

    python3 tools/pmc_traffic.py gpurun_out/pmc_tag profiles/traffic_C2_K128.json
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, dst):
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "pmc_table.py"), src])
    t = json.loads(out)
    full = t["full"]
    fetch = 2.0 * full["FETCH_SIZE"] * 1024.0
    write = full["WRITE_SIZE"] * 1024.0
    res = {"hbm_bytes_per_launch": round(fetch + write),
           "fetch_bytes": round(fetch), "write_bytes": round(write),
           "source": os.path.relpath(src, ROOT),
           "kinds": {k: {c: v for c, v in d.items() if c in ("FETCH_SIZE", "WRITE_SIZE")}
                     for k, d in t.items()},
           "note": "median over the fused launches; FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported"}
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
