"""Print tools/gpu/launch_size.py output: python tools/census_show.py FILE [TOP]"""
import json
import sys

top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for line in open(sys.argv[1]):
    d = json.loads(line)
    print(d["workload"], d["per_launch"], "wall", d["wall_s"], "trials/s", d["trials_per_s"], "end_q_us", d.get("end_q_us"),
          "redo", d["redo_last_chunk"], "ovf", d["stats_0_24"][61] if len(d["stats_0_24"]) > 61 else "-")
    for s in d.get("slowest", [])[:top]:
        print("   ", s)
