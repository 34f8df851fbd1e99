"""Diagnostic: which op issues the activation-sized fills in the update backward?"""
import sys
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
from oc_cleanrl_amd.agents import make_agent  # noqa: E402
from oc_cleanrl_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
ag = make_agent("PPO_OBJ", (4, 12), 6, dev).to(dev)
opt = ops.FlatAdam(ag.parameters(), lr=1e-4, eps=1e-5, max_grad_norm=0.5)
x = torch.randint(0, 160, (4096, 4, 12), device=dev).float()
for it in range(3):
    logits, value = ag.logits_and_value(x)
    if it == 2:
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            torch.autograd.backward([logits, value], [torch.ones_like(logits), torch.ones_like(value)])
            torch.cuda.synchronize()
    else:
        torch.autograd.backward([logits, value], [torch.ones_like(logits), torch.ones_like(value)])
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40))
