"""Soak (scripts/soak.py): burst → delete rounds through one long-lived scheduler with
bind faults and watch drops; the cache, the native HBM ledger and the queue drain after
every round, the cache debugger finds no drift, and the heap stops growing."""
import asyncio
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


def test_soak_rounds_leave_nothing_behind():
    import soak
    res = asyncio.run(soak.soak(rounds=6, pods=300, nodes=4, bind_fail=0.03, drop_watch=700, seed=3,
                                rss_budget_mb=32.0, log=lambda _l: None))
    assert res["ok"], res["problems"]
    rows = res["rounds"]
    assert all(r["bound"] == 300 and r["drained"] and not r["drift"] for r in rows)
    assert rows[-1]["bind_errors"] > 0 and rows[-1]["relists"] > 0        # the faults did fire
    # objects are flat after the first rounds (event buffer bounded, history saturated)
    assert rows[-1]["objects"] - rows[2]["objects"] < 2000, [r["objects"] for r in rows]
    assert res["ledger_size"] == 0
