import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch, icx
from tests.oracle_ffi import smooth, noise
c = icx.Codec(0)
for (h, w) in [(270, 480), (2160, 3840)]:
    imgs = [smooth(h, w, 1), noise(h, w, 2)]
    for target in (10**6 // 4, 2 * 10**6, 16 * 10**6):
        r = c.fit(imgs, target, 0.25)
        print(h, w, target, [(x["success"], x["status"], x["out_len"], x["encodes"], x["learned"]) for x in r], flush=True)
        timgs = [torch.from_numpy(i).cuda() for i in imgs]
        outs = [torch.zeros(target + 1, dtype=torch.uint8, device="cuda") for _ in imgs]
        r = c.fit(timgs, target, 0.25, outputs=outs)
        print("  dev", [(x["success"], x["status"], x["out_len"], x["encodes"]) for x in r], c.last_error(), flush=True)
