"""Debug: bench-shaped decode (B resident C2 batches), histogram of k_decode_st hand-back reasons.

flags bits: 32 BNF_FL_ST, 64 BNF_FL_REDO; debug reasons (k_decode_st): 0x100 sample range,
0x200 truncated, 0x400 padding, 0x800 refill past the CRC point, 0x1000 CRC mismatch.
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from birdnest.audio_amd import libflac, synth

B = int(sys.argv[1]) if len(sys.argv) > 1 else 192
dev = torch.device("cuda:0")
p = synth.config("C2", nframes=1024, seed=2)
s = synth.encode(p)
data = s.data.tobytes()
offs = s.frame_offsets.astype(np.int64)
sp = libflac.StreamParams.from_synth(p, s.nsamples)
copy_len = (len(data) + 255) // 256 * 256
host = np.zeros(copy_len * B + 64, dtype=np.uint8)
for b in range(B):
    host[b * copy_len: b * copy_len + len(data)] = np.frombuffer(data, dtype=np.uint8)
d_bytes = torch.from_numpy(host).to(dev)
d_offs = torch.from_numpy(np.concatenate([offs + b * copy_len for b in range(B)])).to(dev)
nf = 1024 * B
fr_start = np.arange(1024, dtype=np.int64) * p.blocksize
d_os = torch.from_numpy(np.concatenate([fr_start + b * int(s.nsamples) for b in range(B)])).to(dev)
stride = libflac.out_stride(libflac.OUT_FLACDECODER, sp)
d_out = torch.empty(int(s.nsamples) * stride * B, dtype=torch.uint8, device=dev)
d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
dec = libflac.BatchDecoder(0)
dec.decode_frames(d_bytes, copy_len * B, d_offs, nf, sp, libflac.OUT_FLACDECODER, d_out, d_info, d_out_sample=d_os)
torch.cuda.synchronize()
info = libflac.info_array(d_info.cpu().numpy())
h = collections.Counter(int(x) for x in info["flags"])
print("B", B, "flags histogram:", sorted(h.items()))
bad = np.nonzero(info["flags"] & 64)[0]
print("redo frames", len(bad), "first", bad[:10], "frame index in batch", (bad[:10] % 1024))
ok = d_out.cpu().numpy()[: int(s.nsamples) * stride].tobytes() == s.pcm.astype("<i2").tobytes()
print("batch 0 bit-exact", ok, "status all ok", bool((info["status"] == 0).all()), "crc all ok", bool((info["crc_ok"] == 1).all()))
