"""Decode-class mix of one bench config (debug tool): k_parse's routing flags per frame
(k_decode_st / k_decode<8|16|32>), blocksizes per class, and per-class samples, from one
parsed copy of the config's stream.  usage: python tools/class_mix.py C4"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from birdnest.audio_amd import libflac, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
dev = torch.device("cuda:0")
dec = libflac.BatchDecoder(0)
wl = bench.Workload(cfg, 1, None, torch, dev, libflac, synth, dec)
wl.parse(None)
torch.cuda.synchronize()
inf = libflac.info_array(wl.d_info.cpu().numpy())
fl = inf["flags"].astype(np.int64)
bs = inf["blocksize"].astype(np.int64)
cls = np.where(fl & 16, "W32", np.where(fl & 128, "W16", np.where(fl & 32, "ST", "W8")))
tot = bs.sum()
for c in ("ST", "W8", "W16", "W32"):
    m = cls == c
    if m.any():
        print(f"{c:4s} frames {m.sum():6d} samples/ch {bs[m].sum():10d} ({bs[m].sum() / tot:5.1%}) "
              f"bs mean {bs[m].mean():7.0f} max {bs[m].max():6d}")
