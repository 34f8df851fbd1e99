#!/usr/bin/env bash
# Round-5: the mixed tile (56) at imposed splits mbig (rows in 128 x 128 tiles, the rest 64 x 128)
# on the config-2 update shapes, against the 128 x 128 tile (24) and the library's own choice
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mbig
timeout -k 10 200 python3 tools/exp_gemm_x6.py --tiles 24,56 > gpurun_out/mbig/default.jsonl 2>/dev/null
for mb in 3072 4096 5120 6144 7168 8192 9216 10240; do
  timeout -k 10 200 python3 tools/exp_gemm_x6.py --tiles 56 --mbig $mb > gpurun_out/mbig/m$mb.jsonl 2>/dev/null
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/mbig/*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if d.get("kind") in ("fwd", "dx") and d["M"] == 11520:
            print(f.split("/")[-1], d["kind"], d["M"], d["N"], d["K"], {k: v[0] for k, v in d["ours"].items()})
PY
