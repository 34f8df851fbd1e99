"""ppo_loss (prepared records) launch time vs M, to separate the fixed per-launch cost (ticket
fan-in + last-block combine) from the streaming cost."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from tools.kernel_bench import make_case, time_case  # noqa: E402

dev = torch.device("cuda:0")
for M in [65536, 262144, 1 << 20, 2 << 20, 4 << 20, 8 << 20]:
    fn, nbytes = make_case("ppo_loss_prepared", dict(M=M, A=6), dev)
    us = time_case(fn, 10, 5)
    print(json.dumps({"M": M, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
    del fn
    torch.cuda.empty_cache()
