"""Dev probe: whole-model forward error vs the fp64 reference fixture at B=1 and B=32 (the
full_B1_T252 input replicated), under the current K schedules (MST_FORCE_SPLITK to force one)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import detinit  # noqa: E402
from ml_music_style_transfer_amd.model import PerformanceNet  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "full_B1_T252.npz"))
dev = torch.device("cuda", 0)
net = PerformanceNet()
net.load_state_dict({n: torch.from_numpy(detinit.param_value(n, tuple(p.shape)))
                     for n, p in net.named_parameters()})
net = net.to(dev).eval()
x = [torch.from_numpy(a).to(dev) for a in detinit.model_inputs(1, 252)][:3]
idx = torch.from_numpy(g["out_idx"]).to(dev)
y64 = g["out_val64"]
for B in [int(b) for b in sys.argv[1:]] or [1, 2, 4, 8, 16, 32]:
    with torch.no_grad():
        y = net(*(t.expand(B, -1, -1).contiguous() for t in x))
    yv = y.reshape(B, -1)[:, idx].double().cpu().numpy()
    e = np.abs(yv - y64[None]).max()
    r = max(np.linalg.norm(v - y64) / np.linalg.norm(y64) for v in yv)
    print(f"B={B:3d} force_splitk={os.environ.get('MST_FORCE_SPLITK', '0')}: max {e:.3e} rel L2 {r:.3e}",
          flush=True)
