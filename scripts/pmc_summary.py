#!/usr/bin/env python3
"""k_batch PMC ratios from `scripts/gpu_round.sh` step `pmc4` output.

    python scripts/pmc_summary.py gpurun_out/pmc4 [PODS]

Reads `p1_<n>/…counter_collection.csv` and `p2_<n>/…` for n in 256, 1024, 4096 (rocprofv3
`--pmc` passes over `device_batch_bench.py --pods 264 --batch 256`; per pod = per each of the 264), sums each
counter over every k_batch dispatch and prints the ratios kept in `profiles/device/r4/pmc_*`:
waves, VALU active / wave cycles, waiting / wave cycles, LDS bank-conflict / LDS active
cycles, VALU instructions per wave per batch pod."""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def counters(root: str, tag: str) -> dict:
    """Sum per counter over k_batch dispatches: `root/<tag>/…` (gpurun_out) or `root/<tag>_*` (copied)."""
    acc: collections.Counter = collections.Counter()
    paths = glob.glob(os.path.join(root, tag, "**", "*counter_collection.csv"), recursive=True) + \
        glob.glob(os.path.join(root, f"{tag}_*counter_collection.csv"))
    for path in paths:
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if "k_batch" in row["Kernel_Name"]:
                    acc[row["Counter_Name"]] += float(row["Counter_Value"])
    return acc


def main() -> int:
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc4"
    pods = int(sys.argv[2]) if len(sys.argv) > 2 else 264
    print("| nodes | waves | VALU active / wave cycles | waiting / wave cycles | LDS conflict / LDS active | VALU insts per wave per pod |")
    print("|---|---|---|---|---|---|")
    for n in (256, 1024, 4096):
        c = counters(root, f"p1_{n}")
        c.update(counters(root, f"p2_{n}"))
        if not c:
            continue
        waves = c["SQ_WAVES"]
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        lds = c["SQ_ACTIVE_INST_LDS"] or 1.0
        print(f"| {n} | {waves:.0f} | {100 * c['SQ_ACTIVE_INST_VALU'] / wc:.1f} % | "
              f"{100 * c['SQ_WAIT_ANY'] / wc:.1f} % | {c['SQ_LDS_BANK_CONFLICT'] / lds:.2f} | "
              f"{c['SQ_INSTS_VALU'] / max(waves, 1) / pods:.0f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
