"""Debug: FLACDecoder-layout batch decode vs source PCM; first mismatching samples per frame."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from birdnest.audio_amd import libflac, synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "C1"
p = synth.config(cfg, nframes=10, last_blocksize=0)
s = synth.encode(p)
data = s.data.tobytes()
sp = libflac.StreamParams.from_synth(p, s.nsamples)
dev = torch.device("cuda:0")
n = len(data)
d_bytes = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
d_bytes[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
offs = torch.tensor([int(o) for o in s.frame_offsets], dtype=torch.int64, device=dev)
nf = len(s.frame_offsets)
d_out = torch.full((int(s.nsamples) * 4 + 64,), 0xAB, dtype=torch.uint8, device=dev)
d_info = torch.zeros(nf * 128, dtype=torch.uint8, device=dev)
dec = libflac.BatchDecoder(0)
dec.decode_frames(d_bytes, n, offs, nf, sp, libflac.OUT_FLACDECODER, d_out, d_info)
torch.cuda.synchronize()
info = libflac.info_array(d_info.cpu().numpy())
got = d_out.cpu().numpy()[: int(s.nsamples) * 4].view("<u2").reshape(-1, 2)
want = (s.pcm.astype(np.int64) & 0xFFFF).astype("<u2")
bad = np.nonzero((got != want).any(1))[0]
print("flags", info["flags"].tolist(), "status", info["status"].tolist())
print("mismatching samples", len(bad))
for fr in range(nf):
    b = bad[(bad >= fr * 4096) & (bad < (fr + 1) * 4096)] - fr * 4096
    if len(b):
        print("frame", fr, "n", len(b), "first", b[:8].tolist(), "chunks", sorted(set((b // 16).tolist()))[:12])
        i = b[0]
        print("  got", got[fr * 4096 + i: fr * 4096 + i + 4].tolist(), "want", want[fr * 4096 + i: fr * 4096 + i + 4].tolist())
