"""Phase stamps of the heads_loss rows kernel (probe build -DOCPPO_HL_PHASES): per wave the
shader-clock cycles from kernel start to rows done / LDS image synced / record issued.

    python tools/build_variant.py tools/variants/hl_phases.so -DOCPPO_HL_PHASES
    OCPPO_LIB=tools/variants/hl_phases.so python tools/exp_hl_phases.py
"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.kernel_bench import SIZES, make_case  # noqa: E402

dev = torch.device("cuda:0")
for size in ("config", "scaled"):
    p = SIZES["heads_loss"][size]
    fn, _ = make_case("heads_loss", p, dev)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    # make_case's closure owns gp: find it through the closure cells
    gp = next(c.cell_contents for c in fn.__closure__
              if isinstance(c.cell_contents, torch.Tensor) and c.cell_contents.shape == (p["M"], p["H"]))
    fn()
    torch.cuda.synchronize()
    G = min(-(-p["M"] // 16), 256)
    d = gp.view(-1)[:G * 16].view(G, 4, 4).cpu().numpy()
    for i, name in enumerate(("rows done", "LDS synced", "record issued")):
        v = d[:, :, i]
        print(f"{size:7s} {name:14s} cycles: median {np.median(v):9.0f}  p10 {np.percentile(v, 10):9.0f}"
              f"  p90 {np.percentile(v, 90):9.0f}  max {v.max():9.0f}")
    st = d[:, 0, 3]
    print(f"{size:7s} start spread (24-bit clock): {np.ptp(st):.0f} cycles")
