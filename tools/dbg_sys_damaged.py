"""Reproduce test_damaged_and_truncated_identical case by case and print, for the first frame whose
PCM differs between the lane kernels and k_decode_sys, both records' flags / status and the
byte span that differs, under BNFLAC ablate masks given on the command line (default 0 and the
old producer run 0x800000).  usage: python tools/dbg_sys_damaged.py [mask ...]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.test_gpu_decode_sys import FIELDS, _decode, _frame_range, _offsets, _sp  # noqa: E402


def main():
    import torch
    from birdnest.audio_amd import libflac, synth
    L = libflac.load()
    gpu = (torch, libflac, libflac.BatchDecoder(0), L)
    masks = [int(x, 0) for x in sys.argv[1:]] or [0, 0x800000]
    rng = np.random.default_rng(91)
    only = None
    if masks and masks[0] < 0:
        only = -masks[0]
        masks = masks[1:] or [0]
    for i in range(16):
        cfg = ["C1", "C2", "C3", "C4", "C5"][i % 5]
        s = synth.encode(synth.config(cfg, nframes=int(rng.integers(4, 16)), last_blocksize=0, seed=300 + i))
        data = bytearray(s.data.tobytes())
        offs = _offsets(s)
        flips = []
        for _ in range(int(rng.integers(1, 5))):
            p = int(rng.integers(offs[0] + 4, len(data)))
            x = int(rng.integers(1, 256))
            data[p] ^= x
            flips.append((p, x))
        if i % 3 == 2:
            data = data[:len(data) * 3 // 4]
            offs = [o for o in offs if o < len(data)]
        data = bytes(data)
        if only is not None and i != only:
            continue
        sp = _sp(libflac, data)
        fmt = libflac.OUT_INTERLEAVED32
        a, oa, stride = _decode(gpu, data, offs, fmt, False, sp)
        for m in masks:
            L.bnflac_debug_set_ablate(m)
            b, ob, _ = _decode(gpu, data, offs, fmt, True, sp)
            L.bnflac_debug_set_ablate(0)
            rec = [k for k in FIELDS if (a[k] != b[k]).any()]
            bad = []
            for f in np.nonzero(a["status"] == 0)[0]:
                s0, nb = _frame_range(libflac, fmt, a, f, stride)
                d = np.nonzero(oa[s0:s0 + nb] != ob[s0:s0 + nb])[0]
                if len(d):
                    bad.append((int(f), int(d[0]), int(d[-1]), int(len(d)), nb))
            print(f"case {i} {cfg} mask {m:#x} flips {flips} nframes {len(offs)} bytes {len(data)}: "
                  f"records differ {rec} pcm bad {bad[:4]}", flush=True)
            for f, *_ in bad[:2]:
                print(f"   frame {f} off {offs[f]} lane flags {int(a['flags'][f]):#x} sys flags {int(b['flags'][f]):#x} "
                      f"bs {int(a['blocksize'][f])} ch {int(a['channels'][f])} bps {int(a['bps'][f])} "
                      f"as {int(a['assignment'][f])} os {int(a['out_sample'][f])}", flush=True)
                s0, nb = _frame_range(libflac, fmt, a, f, stride)
                key = oa[s0:s0 + 64].tobytes()
                at = ob.tobytes().find(key)
                print(f"   frame's first 64 bytes found in sys output at {at} (frame starts {s0}); "
                      f"other frames' starts {[_frame_range(libflac, fmt, a, g, stride)[0] for g in range(len(offs))]}", flush=True)


if __name__ == "__main__":
    main()
