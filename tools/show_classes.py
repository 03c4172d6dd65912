"""Print the per-class ms/step of a bench.py log line (last line), filtered by substrings."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = sys.argv[2:]
print(d["ms_per_step"], {k: v["ms_per_step"] for k, v in d.get("kernels", {}).items()
                          if not keys or any(s in k for s in keys)})
