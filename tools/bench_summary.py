"""One line per workload of a bench.py JSON line: trials/s, ms per step,
dominant kernel and its roofline fraction, cold start, parity."""
import json
import sys


def line(name, r):
    c = r.get("cold_start", {})
    p = r.get("parity") or {}
    return (f"{name:7s} {r['value']:>12,.0f} trials/s  {r['ms_per_step']:9.2f} ms/step  "
            f"{r['roofline']['kernel']} frac {r['roofline']['frac']:.4f}  "
            f"golden {c.get('golden_s', 0):.2f}s first-step {c.get('first_step_s', 0):.2f}s "
            f"jit-ready {c.get('translated_ready_s', 0):.1f}s  "
            f"parity {p.get('checked')}/{p.get('mismatches')}  esc {r.get('escape_sub')}")


d = json.load(open(sys.argv[1]))
print(line(d["config"]["workload"].split()[0], d))
for n, r in d.get("workloads", {}).items():
    print(line(n, r))
if d.get("cpu_baseline"):
    print("cpu baseline", round(d["cpu_baseline"]["value"]), "trials/s on", d["cpu_baseline"]["cores"], "cores")
