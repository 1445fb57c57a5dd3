#!/usr/bin/env python3
"""Derived per-kernel PMC metrics from tools/pmc_summary.py outputs (one file
per rocprofv3 --pmc pass, counters averaged per dispatch):

    python tools/pmc_derived.py gpurun_out/X/pmc1.txt gpurun_out/X/pmc2.txt [kernel-regex]

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 4 SIMDs / SQ_BUSY_CU_CYCLES
LDS active = SQ_LDS_IDX_ACTIVE / SQ_BUSY_CU_CYCLES
conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
VALU active = SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES (quad-cycle units, as the round-5 files)
wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier)."""
import re
import sys
from collections import defaultdict


def parse(paths):
    k = None
    agg = defaultdict(dict)
    for p in paths:
        for line in open(p):
            if not line.startswith(" ") and line.strip():
                k = line.strip()
            elif line.strip() and k is not None:
                name, val = line.split()
                agg[k][name.replace("SQ_", "")] = float(val)
    return agg


def main():
    files = [a for a in sys.argv[1:] if a.endswith(".txt")]
    pat = re.compile(next((a for a in sys.argv[1:] if not a.endswith(".txt")), "."))
    for k, c in parse(files).items():
        if not pat.search(k) or "BUSY_CU_CYCLES" not in c or c["BUSY_CU_CYCLES"] == 0:
            continue
        cu = c["BUSY_CU_CYCLES"]
        parts = []
        if "VALU_MFMA_BUSY_CYCLES" in c:
            parts.append(f"MFMA busy {100 * c['VALU_MFMA_BUSY_CYCLES'] / 4 / cu:5.1f} %")
        if "LDS_IDX_ACTIVE" in c:
            parts.append(f"LDS active {100 * c['LDS_IDX_ACTIVE'] / cu:5.1f} %")
            if c["LDS_IDX_ACTIVE"] > 0 and "LDS_BANK_CONFLICT" in c:
                parts.append(f"conflict share {100 * c['LDS_BANK_CONFLICT'] / c['LDS_IDX_ACTIVE']:5.1f} %")
        if "ACTIVE_INST_VALU" in c:
            parts.append(f"VALU active {100 * c['ACTIVE_INST_VALU'] / cu:5.1f} %")
        if "WAIT_ANY" in c and c.get("WAVE_CYCLES"):
            parts.append(f"wait {100 * c['WAIT_ANY'] / c['WAVE_CYCLES']:5.1f} %")
        print(f"{k[:40]:<40} " + "  ".join(parts))
        print("    " + "  ".join(f"{n}={v / 1e6:.1f}" for n, v in sorted(c.items())))


if __name__ == "__main__":
    main()
