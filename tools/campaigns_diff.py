#!/usr/bin/env python3
"""Compare the outcome counts of two campaigns summaries (tools/campaigns.py):
python tools/campaigns_diff.py profiles/A_campaigns.json profiles/B_campaigns.json
Prints every configuration whose classes or crash / escape sub-codes differ,
and the trials/s of both."""
import json
import sys

KEYS = ("masked", "sdc", "crash", "hang", "detected", "escape", "crash_sub", "escape_sub")


def ident(r):
    return tuple(str(r.get(k)) for k in ("config", "workload", "structures", "burst", "protect_mask",
                                         "protect_opclasses", "fu_model", "pool"))


a = {ident(r): r for r in json.load(open(sys.argv[1]))}
b = {ident(r): r for r in json.load(open(sys.argv[2]))}
same = 0
for k, rb in b.items():
    ra = a.get(k)
    if ra is None:
        print("new:", k)
        continue
    diff = [x for x in KEYS if ra.get(x) != rb.get(x)]
    if diff:
        print("DIFF", k, {x: (ra.get(x), rb.get(x)) for x in diff})
    else:
        same += 1
    print(f"  {k[0]} {k[1]}: {ra['trials_per_s']:.0f} -> {rb['trials_per_s']:.0f} trials/s")
print(f"{same} of {len(b)} configurations identical")
