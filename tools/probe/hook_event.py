"""Probe: external event record from a post-accumulate-grad hook during graph capture."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "acc-unet-unext_amd"))
import torch
from accunet import kern
lin = torch.nn.Linear(256, 256).cuda()
x = torch.randn(64, 256, device="cuda")
ev = kern.ExtEvent()
info = {}
def hook(p):
    st = torch.cuda.current_stream()
    info["hook_stream"] = st.cuda_stream
    info["capturing"] = torch.cuda.is_current_stream_capturing()
    try:
        ev.record_external()
        info["rec"] = "ok"
    except Exception as e:
        info["rec"] = str(e)
    try:
        ev.record_external(info["cap_stream_obj"])
        info["rec_capstream"] = "ok"
    except Exception as e:
        info["rec_capstream"] = str(e)
h = lin.weight.register_post_accumulate_grad_hook(hook)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    lin(x).sum().backward()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("eager:", info)
lin.weight.grad = None; lin.bias.grad = None
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    info["cap_stream_obj"] = torch.cuda.current_stream()
    info["cap_stream"] = torch.cuda.current_stream().cuda_stream
    lin(x).sum().backward()
print("capture:", {k: v for k, v in info.items() if k != "cap_stream_obj"})
