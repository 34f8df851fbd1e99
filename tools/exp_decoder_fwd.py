"""The update's decoder forward [M x 512] from K = W*E = 2048 (architectures/ppo.py:77-80, the
minibatch forward of ppo_atari_oc.py:566): hipBLASLt's f32 GEMM (+ bias/ReLU epilogue) against
ocppo_gemm_x6 split-K (S partial products + the split combine), device time per call (experiment).

    python tools/exp_decoder_fwd.py > gpurun_out/exp_decoder_fwd.jsonl
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from oc_cleanrl_amd import ops  # noqa: E402
from exp_gemm_x6 import dev_time_us  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M, N, K = 4096, 512, 2048
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.relu(torch.randn(M, K, device=dev, generator=g))
    w = torch.randn(N, K, device=dev, generator=g) * 0.02
    b = torch.randn(N, device=dev, generator=g) * 0.1
    ref = torch.relu(x.double() @ w.double().t() + b.double())
    rec = {"M": M, "N": N, "K": K}
    rec["hipblaslt_us"] = dev_time_us(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False), 20)
    for S in (1, 2, 4, 8):
        for t in list(range(ops.X6_AUTO, ops.X6_AUTO + 4)) + [ops.X6_MIXED]:
            if t == ops.X6_MIXED and S != 1:
                continue
            bm, bn = ops.X6_TILES[t]
            if M % bm or N % bn:
                continue
            part = torch.empty(S, M, N, device=dev)
            out = torch.empty(M, N, device=dev)

            def gemm(S=S, t=t, part=part):
                ops.gemm_x6(x, K, 1, w, K, 1, part, N, M, N, K, splits=S, split_c=M * N, tile=t)

            us = dev_time_us(gemm, 20)
            comb = dev_time_us(lambda part=part, out=out: ops.sum_splits(part, out), 20) if S > 1 else 0.0
            gemm()
            y = torch.relu(part.double().sum(0) + b.double())
            e = float(((y - ref).abs() / ref.abs().max()).max())
            rec[f"x6_s{S}_t{t}"] = {"gemm_us": round(us, 2), "combine_us": round(comb, 2), "err": e}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
