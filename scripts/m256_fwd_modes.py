"""Width-256 decoder forward with and without the training stores (the
activation / mask tiles the weight gradients read): the difference is the
stores' cost inside k_dec256_fwd.  Profile under rocprofv3 --kernel-trace."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo.decoder import Decoder  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 466287
torch.manual_seed(0)
dec = Decoder(depth=2, width=256, in_dim=16, skips=[], embedder="none").cuda()
x = torch.randn(m, 16, device="cuda") * 0.3
for mode in ("train", "infer", "train", "infer"):
    for _ in range(4):
        if mode == "train":
            out = dec({"emb": x.requires_grad_(True)})
        else:
            with torch.no_grad():
                out = dec({"emb": x.detach()})
    torch.cuda.synchronize()
    print(mode, "done")
