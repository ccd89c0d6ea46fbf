"""Run native conv fwd / dgrad / wgrad on every eligible conv shape of the given zoo models (batch 128)
and report the ones the launchers reject.  python tools/probe_conv_shapes.py DPN26 ..."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.models import build_model  # noqa: E402
from fedmi.ops import conv as C  # noqa: E402
from fedmi.ops import native_mode as nm  # noqa: E402

dev = torch.device("cuda", 0)
for name in sys.argv[1:]:
    m = build_model(name)
    shapes = set()
    hooks = [mm.register_forward_hook(lambda mod, i, o: shapes.add(
        (tuple(i[0].shape[1:]), mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0]))
        if isinstance(mod, torch.nn.Conv2d) and nm._conv_kind(mod.in_channels, mod.out_channels, mod.groups,
                                                                mod.kernel_size, mod.stride, mod.padding,
                                                                mod.dilation) == "mfma" else None)
        for mm in m.modules()]
    m(torch.randn(2, 3, 32, 32))
    for (c, h, w), O, k, st, pad in sorted(shapes):
        x = torch.randn(128, h, w, c, device=dev).bfloat16()
        wt = torch.randn(O, c, k, k, device=dev) * 0.05
        res = {"model": name, "shape": [c, h, O, k, st, pad]}
        for op in ("fwd", "dgrad", "dgrad_tap", "wgrad"):
            try:
                wp = C.pack_weight(wt)
                if op == "fwd":
                    C.conv2d_fwd(x, wp, st, pad, ws=C.wgrad_workspace(dev, C.fd_ws_floats(x.shape, O, k, k, st, pad)))
                else:
                    P, Q = C.out_hw(h, w, k, k, st, pad)
                    dy = torch.randn(128, P, Q, O, device=dev).bfloat16()
                    if op == "wgrad":
                        C.conv2d_wgrad(x, dy, k, k, st, pad)
                    elif op == "dgrad":
                        C.conv2d_dgrad(dy, wp, x.shape, st, pad)
                    elif C.dgrad_eligible(O):
                        wd = torch.empty(C.dgrad_image_numel(wt.shape), dtype=torch.bfloat16, device=dev)
                        C.dgrad_pack_weights([(wt, wd, st, pad, c)])
                        C.conv2d_dgrad(dy, wp, x.shape, st, pad, wd=wd)
                torch.cuda.synchronize()
                res[op] = "ok"
            except Exception as e:  # launch-config rejections only (host-side errors)
                res[op] = str(e)[:120]
        print(json.dumps(res), flush=True)
