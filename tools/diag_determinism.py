"""Native mode: run the same training forward/backward twice and report the first module whose
output (and the parameters whose gradient) differ between the runs."""
import copy
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fedmi.models import build_model  # noqa: E402
from fedmi.ops.native_mode import NativeMode  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "SimpleDLA"
dev = torch.device("cuda", 0)
torch.manual_seed(0)
base = build_model(name).to(dev)
x = torch.randn(128, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last).bfloat16()
y = torch.randint(0, 10, (128,), device=dev)


def run():
    m = copy.deepcopy(base)
    m.train()
    outs = {}
    hooks = [mod.register_forward_hook(lambda mod, i, o, n=n: outs.__setitem__(n, (type(mod).__name__, o.detach().float().clone())))
             for n, mod in m.named_modules() if n]
    with NativeMode(strict=True):
        loss = F.cross_entropy(m(x), y)
        loss.backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    return outs, {n: p.grad.clone() for n, p in m.named_parameters()}, float(loss)


a_out, a_g, la = run()
b_out, b_g, lb = run()
print("loss", la, lb)
shown = 0
for n, (t, v) in a_out.items():
    d = float((v - b_out[n][1]).abs().max())
    if d > 0 and shown < 8:
        print(f"fwd diff {n} ({t}) shape={tuple(v.shape)}: {d:.4g} (max {float(v.abs().max()):.4g})")
        shown += 1
print("first-differing forward outputs shown:", shown)
worst = sorted(((float((a_g[n] - b_g[n]).abs().max() / (a_g[n].abs().max() + 1e-12)), n) for n in a_g), reverse=True)[:8]
for d, n in worst:
    print(f"grad rel diff {n}: {d:.4g}")

# fp32 PyTorch reference gradients (same weights, same bf16-valued input) and bf16 autocast PyTorch
m = copy.deepcopy(base)
m.train()
F.cross_entropy(m(x.float()), y).backward()
ref = {n: p.grad.clone() for n, p in m.named_parameters()}
m = copy.deepcopy(base)
m.train()
with torch.autocast("cuda", dtype=torch.bfloat16):
    lo = F.cross_entropy(m(x.float().contiguous(memory_format=torch.channels_last)), y)
lo.backward()
ac = {n: p.grad.clone() for n, p in m.named_parameters()}


def rel(g, n):
    return float((g[n] - ref[n]).abs().max() / (ref[n].abs().max() + 1e-12))


worst = sorted(((rel(a_g, n), n) for n in ref), reverse=True)[:6]
for d, n in worst:
    print(f"vs fp32 {n}: native-a {d:.4g} native-b {rel(b_g, n):.4g} autocast-bf16 {rel(ac, n):.4g}")
tot = lambda g: float(torch.cat([(g[n] - ref[n]).flatten() for n in ref]).norm() / torch.cat([ref[n].flatten() for n in ref]).norm())  # noqa: E731
print(f"global grad rel-L2 vs fp32: native-a {tot(a_g):.4g} native-b {tot(b_g):.4g} autocast-bf16 {tot(ac):.4g}")
