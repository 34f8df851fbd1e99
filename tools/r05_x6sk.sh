#!/usr/bin/env bash
# Round-5: gemm_x6 pipelined tiles, plain / stream-K / pre-split B, config-2 shapes
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
show() {
  python3 - "$1" "$2" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    r = json.loads(ln)
    if r["kind"] == "total":
        continue
    print(sys.argv[2], r["kind"], r["M"], r["N"], r["K"], " ".join(f"{t}:{v[0]}/{v[2][0]:.1e}" for t, v in r["ours"].items()))
PY
}
timeout -k 10 400 python3 tools/exp_gemm_x6.py --tiles 24,56,57,58 --reps 20 --stream-k --out gpurun_out/x6sk_sk.jsonl > gpurun_out/x6sk_sk.log 2>&1
show gpurun_out/x6sk_sk.jsonl sk
timeout -k 10 400 python3 tools/exp_gemm_x6.py --tiles 24,56,57,58 --reps 20 --stream-k --planes --out gpurun_out/x6sk_skpl.jsonl > gpurun_out/x6sk_skpl.log 2>&1
show gpurun_out/x6sk_skpl.jsonl skpl
