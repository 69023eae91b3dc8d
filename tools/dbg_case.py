"""Debug one synthetic stream: per-frame GPU vs source PCM, with the frame records."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from birdnest.audio_amd import libflac, synth

kw = json.loads(sys.argv[1])
ablate = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
s = synth.encode(synth.config("C2", **kw))
data = s.data.tobytes()
sp = libflac.StreamParams.from_synth(s.params, s.nsamples)
dev = torch.device("cuda:0")
nb = len(data)
d_bytes = torch.zeros((nb + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
d_bytes[:nb] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
offs = torch.from_numpy(s.frame_offsets.astype(np.int64)).to(dev)
nf = len(s.frame_offsets)
C = s.pcm.shape[1]
d_out = torch.zeros(int(s.nsamples) * 4 * C + 64, dtype=torch.uint8, device=dev)
d_info = torch.zeros(nf * 128, dtype=torch.uint8, device=dev)
dec = libflac.BatchDecoder(0)
if ablate:
    dec.L.bnflac_debug_set_ablate(ablate)
dec.decode_frames(d_bytes, nb, offs, nf, sp, libflac.OUT_INTERLEAVED32, d_out, d_info)
torch.cuda.synchronize()
info = libflac.info_array(d_info.cpu().numpy())
out = d_out.cpu().numpy()[: int(s.nsamples) * 4 * C].view("<i4").reshape(-1, C)
nbad = 0
for fr in range(nf):
    st, b = int(info["out_sample"][fr]), int(info["blocksize"][fr])
    g, w = out[st: st + b], s.pcm[st: st + b]
    if not np.array_equal(g, w):
        nbad += 1
        if nbad <= 4:
            rows = np.nonzero((g != w).any(1))[0]
            cols = np.nonzero((g != w).any(0))[0]
            print("frame", fr, "bs", b, "status", int(info["status"][fr]), "crc_ok", int(info["crc_ok"][fr]), "flags",
                  int(info["flags"][fr]), "bad rows", len(rows), "first", rows[:6].tolist(), "channels", cols.tolist(),
                  "sub_start", info["sub_start"][fr][:C].tolist())
            r = rows[0]
            print("   got", g[r:r + 3].tolist(), "want", w[r:r + 3].tolist())
print("frames", nf, "bad", nbad)
for fr in np.nonzero(info["status"] != 0)[0][:4]:
    print("status!=0 frame", int(fr), "status", int(info["status"][fr]), "err", int(info["err"][fr]), "flags",
          int(info["flags"][fr]), "bs", int(info["blocksize"][fr]), "resume_bit", int(info["resume_bit"][fr]),
          "frame_off", int(info["frame_off"][fr]), "next_off", int(s.frame_offsets[fr + 1]) if fr + 1 < nf else nb,
          "sub_start", info["sub_start"][fr][:C].tolist(), "crc_ok", int(info["crc_ok"][fr]))
np.save("gpurun_out/dbg_info.npy", d_info.cpu().numpy())
