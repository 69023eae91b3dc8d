"""Debug: compare k_decode_st + hand-back against k_decode<8> alone on one config."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tests import test_gpu_parity as T
from birdnest.audio_amd import libflac, synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
gpu = (torch, libflac, libflac.BatchDecoder(0))
p = synth.config(cfg, nframes={"C4": 64}.get(cfg, 16), last_blocksize=0)
s = synth.encode(p)
data = s.data.tobytes()
fmt = getattr(libflac, sys.argv[2] if len(sys.argv) > 2 else "OUT_FLACDECODER")
out_a, ia, _ = T._decode_batch(gpu, data, s.frame_offsets, fmt)
gpu[2].L.bnflac_debug_set_ablate(0x400)
out_b, ib, _ = T._decode_batch(gpu, data, s.frame_offsets, fmt)
gpu[2].L.bnflac_debug_set_ablate(0)
d = np.nonzero(out_a != out_b)[0]
print("ndiff", len(d), "first", d[:8])
for f in range(len(ia)):
    o0, bs = int(ia["out_sample"][f]) * 4, int(ia["blocksize"][f]) * 4
    nd = int(((d >= o0) & (d < o0 + bs)).sum())
    if nd or f < 3:
        print(f, "st", ia["status"][f], ib["status"][f], "flags", ia["flags"][f], ib["flags"][f], "bs", ia["blocksize"][f],
              "os", ia["out_sample"][f], "as", ia["assignment"][f], "crc", ia["crc_ok"][f], ib["crc_ok"][f], "nd", nd)
import collections
print("flags histogram (ST run):", collections.Counter(int(x) for x in ia["flags"]))
