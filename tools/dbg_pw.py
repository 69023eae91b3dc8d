#!/usr/bin/env python3
"""Debug: k_parse_wave on one frame of a golden fixture (BNFLAC_LIB_DIR=<variant dir>)."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from birdnest.audio_amd import libflac
G = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
name, off = sys.argv[1], int(sys.argv[2])
data = open(os.path.join(ROOT, "tests/golden", G[name]["file"]), "rb").read()
si = data[8:42]
x = int.from_bytes(si[10:18], "big")
sp = libflac.StreamParams(1, int.from_bytes(si[0:2], "big"), int.from_bytes(si[2:4], "big"), x >> 44,
                          ((x >> 41) & 7) + 1, ((x >> 36) & 31) + 1, x & ((1 << 36) - 1))
L = libflac.load()
dec = libflac.BatchDecoder(0)
dev = torch.device("cuda:0")
d_bytes = torch.zeros((len(data) + 15) // 16 * 16 + 32, dtype=torch.uint8, device=dev)
d_bytes[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
d_offs = torch.tensor([off], dtype=torch.int64, device=dev)
for mode in (0, 1):
    d_info = torch.zeros(libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    L.bnflac_debug_set_parse_wave(mode)
    dec.parse_frames(d_bytes, len(data), d_offs, 1, sp, d_info)
    torch.cuda.synchronize()
    print("mode", mode, libflac.info_array(d_info.cpu().numpy())[0], flush=True)
