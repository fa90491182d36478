#!/usr/bin/env python3
"""Summarise a gpu_ab.py JSONL (bench.py rows) per variant: pods/s, p99, CPU/pod, reset, thread CPU."""
import collections
import json
import statistics as S
import sys


def main(path: str) -> None:
    rows = [json.loads(line) for line in open(path)]
    by, order = collections.defaultdict(list), []
    for r in rows:
        if r["variant"] not in order:
            order.append(r["variant"])
        by[r["variant"]].append(r)
    for v in order:
        rs = by[v]
        med = lambda k: S.median(x[k] for x in rs if x.get(k) is not None)  # noqa: E731
        th = collections.defaultdict(list)
        for x in rs:
            for k, val in (x.get("thread_cpu_us_per_pod") or {}).items():
                th[k].append(val)
        eng = [x["lane_engine_us_per_pod"]["cpu"] for x in rs if x.get("lane_engine_us_per_pod")]
        vals = " ".join("%.1fk" % (x["value"] / 1e3) for x in rs)
        print(f"{v:10s} pods/s {vals} (median {med('value') / 1e3:.1f}k) | "
              f"p99 {med('p99_latency_ms'):.3f} | cpu/pod {med('cpu_us_per_pod'):.2f} | "
              f"reset {med('reset_ms_median'):.3f} | threads {dict((k, S.median(x)) for k, x in th.items())} | "
              f"engine {S.median(eng) if eng else None}")


if __name__ == "__main__":
    main(sys.argv[1])
