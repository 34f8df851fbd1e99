"""Print a bench line's value and its top in-graph kernel sites: python tools/show_line.py FILE [N]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"])
ks = d.get("kernels", {})
for k, v in sorted(ks.items(), key=lambda kv: -(kv[1].get("us_per_iter") or 0))[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print(f"  {k:40s} {v.get('mean_us')!s:>10} x {v.get('launches_per_iter')!s:>4} = {v.get('us_per_iter')}")
