#!/usr/bin/env python3
"""HIP / HSA API census of a ``rocprofv3 --hip-trace --hsa-trace --stats`` run: calls and time
per API (from the *_api_stats.csv files) and calls per thread per API (from the traces), so the
host CPU a device-mode scheduler spends in the ROCm runtime can be attributed to call sites.
The raw trace CSVs are deleted afterwards (they can be large); the stats and this census stay.

    python scripts/api_census.py gpurun_out/hiptrace6 [--keep]
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def main(argv: list[str]) -> int:
    root = argv[0]
    keep = "--keep" in argv
    for stats in sorted(glob.glob(os.path.join(root, "**", "*api_stats.csv"), recursive=True)):
        print(f"== {os.path.relpath(stats, root)}")
        rows = list(csv.DictReader(open(stats)))
        rows.sort(key=lambda r: -float(r.get("TotalDurationNs") or 0))
        for r in rows[:25]:
            print(f"  {r['Name'][:48]:48s} calls={int(r['Calls']):>9d} total_ms={float(r['TotalDurationNs']) / 1e6:10.3f}"
                  f" avg_us={float(r['AverageNs']) / 1e3:9.3f}")
    for tr in sorted(glob.glob(os.path.join(root, "**", "*api_trace.csv"), recursive=True)):
        by = collections.Counter()
        dur = collections.Counter()
        for r in csv.DictReader(open(tr)):
            k = (r.get("Thread_Id", "?"), r.get("Function", "?"))
            by[k] += 1
            dur[k] += int(r.get("End_Timestamp", 0) or 0) - int(r.get("Start_Timestamp", 0) or 0)
        threads = collections.Counter()
        for (t, _f), n in by.items():
            threads[t] += n
        print(f"== {os.path.relpath(tr, root)}: {sum(by.values())} calls on {len(threads)} threads")
        for t, n in threads.most_common(8):
            top = sorted(((n2, f) for (t2, f), n2 in by.items() if t2 == t), reverse=True)[:8]
            print(f"  thread {t}: {n} calls; " + ", ".join(f"{f}×{n2} ({dur[(t, f)] / 1e6:.1f} ms)" for n2, f in top))
        if not keep:
            os.remove(tr)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
