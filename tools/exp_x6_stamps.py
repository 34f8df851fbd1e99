"""Per-workgroup phase stamps of a pipelined gemm_x6 launch (probe build -DOCPPO_X6_STAMPS):
prologue (loads + first stash), K loop, epilogue (stores drained), and the launch's span on the
real-time clock.

    python tools/build_variant.py tools/variants/x6_stamps.so --only ocppo_gemm.hip -DOCPPO_X6_STAMPS
    OCPPO_LIB=tools/variants/x6_stamps.so python tools/exp_x6_stamps.py --tile 58 --shape dx,4096,512,2048
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=58)
    ap.add_argument("--shape", default="dx,4096,512,2048")
    a = ap.parse_args()
    kind, M, N, K = a.shape.split(",")
    M, N, K = int(M), int(N), int(K)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    if kind == "fwd":
        x = torch.rand(M, K, device=dev, generator=g)
        w = torch.rand(N, K, device=dev, generator=g)
        out = torch.empty(M, N, device=dev)
        fn = lambda: ops.gemm_x6(x, K, 1, w, K, 1, out, N, M, N, K, tile=a.tile)  # noqa: E731
        rows, cols = M, N
    else:
        gg = torch.rand(M, N, device=dev, generator=g)
        w = torch.rand(N, K, device=dev, generator=g)
        out = torch.empty(M, K, device=dev)
        fn = lambda: ops.gemm_x6(gg, N, 1, w, 1, K, out, K, M, K, N, tile=a.tile)  # noqa: E731
        rows, cols = M, K
    bm, bn = ops.X6_TILES[a.tile]
    grid = (rows // bm) * (cols // bn)
    st = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
    setter = _lib.LIB.ocppo_x6_probe_set_stamps
    setter.argtypes = [ctypes.c_void_p]
    for _ in range(3):
        fn()
    setter(st.data_ptr())
    fn()
    torch.cuda.synchronize()
    setter(None)
    d = st.view(grid, 8).cpu().numpy().astype(np.float64)
    pro, loop, epi = d[:, 1] - d[:, 0], d[:, 2] - d[:, 1], d[:, 3] - d[:, 2]
    span_us = (d[:, 5].max() - d[:, 4].min()) / 100.0
    total = d[:, 3] - d[:, 0]
    clk = total.mean() / ((d[:, 5] - d[:, 4]).mean() / 100.0) / 1e3  # cycles per us -> GHz
    for name, v in (("prologue", pro), ("K loop", loop), ("epilogue", epi), ("total", total)):
        print(f"{name:9s} cycles: median {np.median(v):9.0f}  p10 {np.percentile(v, 10):9.0f}  "
              f"p90 {np.percentile(v, 90):9.0f}  max {v.max():9.0f}")
    print(f"start spread {(d[:, 4].max() - d[:, 4].min()) / 100:.2f} us, span {span_us:.2f} us, "
          f"shader clock ~{clk:.2f} GHz, {grid} workgroups, K steps {K // 32}")


if __name__ == "__main__":
    main()
