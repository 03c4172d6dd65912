"""Summarise a bench.py JSON line: headline, forward, roofline, per-class table, extra points."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"value {d['value']} faces/s  {d['ms_per_step']} ms/step  dtype {d['dtype']}  fwd {d.get('forward')}")
r = d.get("roofline")
if r:
    print(f"roofline {r['kernel']}: {r['us_per_launch']} us/launch frac {r['frac']} traffic {r.get('traffic')}")
for k, v in d.get("kernels", {}).items():
    print(f"  {k:30s} {v['ms_per_step']:7.4f} ms x{v['launches']:<3d} mfma {v['mfma_frac']:.3f} hbm {v['hbm_frac']:.3f}"
          + (f" pmc/alg {v['pmc_over_algorithmic']}" if v.get("pmc_over_algorithmic") else ""))
if "same_workload_as_multi_gpu" in d:
    x = d["same_workload_as_multi_gpu"]
    print(f"1M gallery (N=1): {x['value']} faces/s {x['ms_per_step']} ms/step")
if "cpu_baseline" in d:
    print("cpu_baseline", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
