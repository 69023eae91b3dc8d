#!/usr/bin/env python3
"""Experiment: does grouping similar frames into the same wave speed up the generic decode
kernels (k_decode<8|32>, lane per subframe)?  Frame order only decides which frames share a
wave -- output positions come from d_out_sample -- so the host can reorder (offset, position)
pairs.  usage: python tools/exp_sort.py C4 [B]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def sub_types(data, info, nf):
    """(type code, order) of every subframe of the first nf frames from the header bytes."""
    out = []
    for f in range(nf):
        fo = int(info["frame_off"][f]) * 8
        row = []
        for c in range(int(info["channels"][f])):
            bit = fo + int(info["sub_start"][f][c])
            byte, sh = bit >> 3, bit & 7
            x = ((data[byte] << 8 | data[byte + 1]) >> (8 - sh)) & 0xFF
            t = (x >> 1) & 0x3F
            row.append(t)
        out.append(row)
    return out


def main():
    import torch
    from birdnest.audio_amd import libflac, synth
    cfg = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else bench.CONFIGS[cfg]["batches"]
    dev = torch.device("cuda:0")
    dec = libflac.BatchDecoder(0)
    stream = torch.cuda.current_stream(dev)
    wl = bench.Workload(cfg, B, 0, torch, dev, libflac, synth, dec)
    el, tp, td = bench.timed(wl, 3, 1, stream, 1, None, dev)
    print(cfg, "orig   step ms", round(el / 3 * 1e3, 3), "parse", round(tp, 3), "decode", round(td, 3), "ok", wl.check())
    info = libflac.info_array(wl.d_info.cpu().numpy())
    types = sub_types(np.frombuffer(wl.data, dtype=np.uint8), info, wl.nf1)

    def cls(t):  # 0 const, 1 verb, 2 fixed, 3 lpc<=8, 4 lpc<=16, 5 lpc<=32
        if t == 0:
            return 0
        if t == 1:
            return 1
        if 8 <= t <= 12:
            return 2
        o = (t & 31) + 1
        return 3 if o <= 8 else (4 if o <= 16 else 5)
    key1 = np.array([(max(cls(t) for t in row) * 16 + min(cls(t) for t in row)) for row in types])
    bs = info["blocksize"][: wl.nf1].astype(np.int64)
    offs = wl.d_offs.cpu().numpy()
    os_ = wl.d_os.cpu().numpy()
    for name, key in (("by bs", bs), ("by class,bs", key1 * 65536 + bs), ("by bs,class", bs * 64 + key1)):
        kk = np.tile(key, B)
        perm = np.argsort(kk, kind="stable")
        wl.d_offs = torch.from_numpy(offs[perm].copy()).to(dev)
        wl.d_os = torch.from_numpy(os_[perm].copy()).to(dev)
        el, tp, td = bench.timed(wl, 3, 1, stream, 1, None, dev)
        print(cfg, name.ljust(12), "step ms", round(el / 3 * 1e3, 3), "parse", round(tp, 3), "decode", round(td, 3),
              "ok", wl.check())


if __name__ == "__main__":
    main()
