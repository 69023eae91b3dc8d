"""Debug: k_decode_sw line flush on a small C3 batch: where does the FILEREADER output differ?"""
import numpy as np
from tests.test_gpu_parity import _decode_batch
from tests.test_gpu_decode_sw import _expect
import torch
from birdnest.audio_amd import libflac, synth
gpu = (torch, libflac, libflac.BatchDecoder(0))
p = synth.config("C3", nframes=24, last_blocksize=0)
s = synth.encode(p)
out, info, sp = _decode_batch(gpu, s.data.tobytes(), s.frame_offsets, libflac.OUT_FILEREADER)
exp = np.frombuffer(_expect(libflac, libflac.OUT_FILEREADER, s.pcm, info, 24), dtype=np.uint8)
bad = np.nonzero(out != exp)[0]
print("flags", set(info["flags"].tolist()), "status", set(info["status"].tolist()), "bad bytes", len(bad), "of", len(out))
fb = 8192 * 6
for b in bad[:1]:
    print("first bad byte", b, "frame", b // fb, "chunk", (b % fb) // 192, "byte in chunk", (b % fb) % 192)
fr = bad // fb
ch = (bad % fb) // 192
ln = ((bad % fb) % 192) // 64
import collections
print("frames", sorted(collections.Counter(fr.tolist()).items())[:30])
print("chunks", sorted(collections.Counter(ch.tolist()).items())[:12])
print("lines", sorted(collections.Counter(ln.tolist()).items()))
print("unwritten (0xAB) bad bytes", int((out[bad] == 0xAB).sum()))
